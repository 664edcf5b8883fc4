"""Batched bwd-data weight operands: one launch per step instead of two torch kernels per convolution.

The narrow bwd-data kernels (kernels/convn.hip) run dX as a convolution of dY with a re-laid weight
W'[ci][r'][s'][co] = W[co][r0 + r' sr][s0 + s' ss][ci]:

* ``"t"``: a 1x1 convolution's transpose W^T (``w.t().contiguous()``);
* ``"f"``: a stride-1 3x3's tap flip (``w.flip(2, 3).permute(1, 2, 3, 0)``);
* ``"p"``: a stride-2 3x3's four output-parity phase subsets (``conv._s2_phase_weights``).

Built per convolution inside its backward these were ~56 flip / copy launches (~0.45 ms) per
ResNet-50 b1024 step (``profiles/r5/resnet50_b1024_r5n_kernels.md``). Each convolution's forward
registers its operand here (``note``) and marks the device's operands stale; the first backward that
asks for one (``get``) refreshes every registered operand of that device in one ``wprep_run``
launch (kernels/wprep.hip) over a job table that stays on the device. A forward always precedes the
backward that uses its weights, so a backward never sees an operand older than its forward; weights
change only between steps (the PS apply), never between a layer's forward and its backward.

The reference has no counterpart (its worker's compute is a stub, ``/root/reference/src/worker.cpp:316-329``).
"""
from __future__ import annotations

import weakref

import torch

from ..utils.config import feature as _feat


def _geo(kind: str, k: int) -> list:
    """[(Rp, Sp, r0, s0, sr, ss)] of the operands of one kind (several for "p")."""
    if kind == "t":
        return [(1, 1, 0, 0, 1, 1)]
    if kind == "f":
        return [(k, k, k - 1, k - 1, -1, -1)]
    # "p": r in (1,) for ph = 0, (2, 0) for ph = 1; columns alike; phase order ph << 1 | pw
    sel = ((1, 1, 1), (2, 2, -2))  # (count, first, step)
    out = []
    for ph in (0, 1):
        for pw in (0, 1):
            (rc, r0, sr), (sc, s0, ss) = sel[ph], sel[pw]
            out.append((rc, sc, r0, s0, sr, ss))
    return out


class _Entry:
    __slots__ = ("mod", "weight", "shape", "device", "seen", "kind", "geo", "dsts")

    def __init__(self, mod, weight, kind):
        cout, cin, k, _ = weight.shape
        self.mod = weakref.ref(mod)
        self.weight = weakref.ref(weight)  # the Parameter: its storage may alternate (PS double buffer)
        self.shape = tuple(weight.shape)
        self.device = weight.device
        self.seen = {weight.data_ptr()}
        self.kind = kind
        self.geo = _geo(kind, k)
        self.dsts = [torch.empty(cin, rp * sp * cout, device=weight.device, dtype=weight.dtype)
                     for rp, sp, *_ in self.geo]


class _Registry:
    def __init__(self):
        self.entries: dict = {}    # (id(mod), kind) -> _Entry
        self.tables: dict = {}     # device -> {weight storage pointers: (table, tiles)}
        self.stale: dict = {}      # device -> True when a forward ran since the last refresh
        self.volatile: set = set() # keys whose weight storage kept moving: not batched

    def clear(self):
        self.entries.clear()
        self.tables.clear()
        self.stale.clear()
        self.volatile.clear()

    def note(self, mod, weight: torch.Tensor, kind: str) -> None:
        if mod is None or not _feat("wprep") or not _eligible(weight):
            return
        key = (id(mod), kind)
        if key in self.volatile:
            return
        e = self.entries.get(key)
        if e is None or e.mod() is not mod or e.weight() is not weight or e.shape != tuple(weight.shape):
            if torch.cuda.is_current_stream_capturing():
                return  # no new persistent buffers inside a graph capture (its backward builds the operand)
            self.entries[key] = _Entry(mod, weight, kind)
            self.tables.pop(weight.device, None)
        else:
            p = weight.data_ptr()
            if p not in e.seen:
                e.seen.add(p)
                if len(e.seen) > 4:  # a storage re-made every step (not a buffer set): build it in backward
                    self.volatile.add(key)
                    self.entries.pop(key)
                    self.tables.pop(weight.device, None)
                    return
        self.stale[weight.device] = True

    def get(self, mod, weight: torch.Tensor, kind: str):
        """The refreshed operand(s) of ``mod``'s weight (a list of 4 for "p"), or None when the
        forward did not register it (the caller builds it with torch ops)."""
        if mod is None:
            return None
        e = self.entries.get((id(mod), kind))
        if e is None or e.mod() is not mod:
            return None
        w = e.weight()
        if w is None or w.data_ptr() != weight.data_ptr() or e.shape != tuple(weight.shape):
            return None
        dev = weight.device
        if self.stale.get(dev, True) and not self._refresh(dev):
            return None
        return e.dsts if kind == "p" else e.dsts[0]

    def _refresh(self, dev) -> bool:
        """One launch over every registered operand of ``dev``, from the weights' current storage
        (a job table per storage set: the PS's two alternating parameter buffers give two). False
        when a new table would be needed inside a graph capture (its host-to-device upload cannot be
        captured): the callers then build their operands with torch ops."""
        from .. import native

        C = native()
        live, dead = [], False
        for key, e in self.entries.items():
            if e.device != dev:
                continue
            # strong references for the rest of the refresh: a weak reference can die between two
            # dereferences when a collection runs in between (a freed model's entries)
            m, w = e.mod(), e.weight()
            if m is None or w is None:
                dead = True
                continue
            live.append((key, e, w))
        if dead:
            self.entries = {k: e for k, e in self.entries.items() if e.mod() is not None and e.weight() is not None}
            self.tables.pop(dev, None)
        cache = self.tables.setdefault(dev, {})
        sig = tuple(w.data_ptr() for _, _, w in live)
        tab = cache.get(sig)
        if tab is None:
            if torch.cuda.is_current_stream_capturing():
                return False
            if len(cache) >= 4:
                cache.clear()
            srcs, dsts, geo = [], [], []
            for _, e, w in live:
                for d, g in zip(e.dsts, e.geo):
                    srcs.append(w)
                    dsts.append(d)
                    geo.extend(g)
            tab = C.wprep_table(srcs, dsts, geo) if srcs else (None, 0)
            cache[sig] = tab
        if tab[0] is not None:
            C.wprep_run(tab[0], tab[1])
        self.stale[dev] = False
        return True


def _eligible(weight: torch.Tensor) -> bool:
    cout, cin = weight.shape[0], weight.shape[1]
    return (weight.is_cuda and weight.dtype == torch.bfloat16 and weight.dim() == 4 and cout % 8 == 0
            and cin % 8 == 0 and weight.is_contiguous(memory_format=torch.channels_last))


REGISTRY = _Registry()
note = REGISTRY.note
get = REGISTRY.get
