"""Per-shape choice between implementations of one op, timed once with HIP events.

The role MIOpen's Find plays for convolutions, for the places where this framework has both a
hand-written gfx950 kernel and a library path (hipBLASLt / MIOpen) for the same math: the first
eager call of a shape times every candidate (one warm call, then the best of two batches of 3
timed calls), caches the fastest and
uses it from then on. Inside a hipGraph capture nothing is timed: an undecided shape takes the
``default`` candidate (the Trainer always runs eager warmup steps before it captures).

Across ranks (torch.distributed initialised, world > 1) every rank runs the same choice: the first
rank to reach a key claims it through the rendezvous store (an atomic ``add``), times and validates
the candidates and publishes the winner; every other rank waits for that decision instead of
timing on its own. Independent per-rank timing picked different kernels on different ranks (3
timed reps are noisy), so the ranks' step times and numerics differed and the SSP bound tied
everyone to the slowest rank's choices. ``PSD_AUTOTUNE_FILE``: a JSON file of decisions
(``save_decisions``) loaded at import, which pins every listed key on every rank with no timing.
``source()`` reports which of these decided.

Like MIOpen's Find, a candidate must also be *correct* to be chosen: the outputs of its warm call
and of its last timed call are compared with the default candidate's (finite wherever the default
is finite, max |diff| <= 3 % of max |ref|, no absolute floor). A library solution that returns garbage is dropped.
This is not hypothetical: the hipBLASLt solution TunableOp had recorded for ResNet-50's
layer1 conv3 forward (``tn_256_3211264_64``, b1024) returned NaN/garbage rows, the timing-based
choice picked it on some runs, and the BN ReLU turned the NaN into zeros so the step kept a
finite loss on broken weights (tools/rank_check.py, tools/gemm_nan_probe.py; README).
"""
from __future__ import annotations

import ast
import datetime
import json
import os
import time

import torch

from ..utils.config import feature as _feat

_DECISIONS: dict[tuple, str] = {}
_DECLINED_KEYS: set = set()  # keys where every candidate declined (decided once, for every rank)
_DECLINED = "__declined__"
_FAILED = "__failed__"
_SOURCE = {"local": 0, "claimed": 0, "peer": 0, "file": 0}
_FILE_KEYS: set = set()


_REJECTED: dict[tuple, list] = {}


class Declined(RuntimeError):
    """Raised by a candidate whose kernel does not take this shape. While a key is being timed
    the candidate is simply left out (recorded in ``rejected()`` as "declined:<name>"); a candidate
    that was chosen and then declines is an error -- never a silent switch to another kernel
    behind the recorded decision."""
_TIMES: dict[tuple, dict] = {}


def _snap(out, probe):
    if out is None and probe is not None:
        out = probe()
    return out.detach().float().clone() if isinstance(out, torch.Tensor) else None


def _time_ms(fn, reps: int = 3, probe=None, batches: int = 2):
    """(ms per call, [output of the warm call, output of the last timed call]): the best of
    ``batches`` batch means of ``reps`` calls each. One batch of 3 let a clock / interference blip
    flip close decisions from run to run (ResNet-50: ~1 ms/step of kernel choices moved between two
    same-box runs, profiles/r5/)."""
    outs = [_snap(fn(), probe)]  # warm (library heuristics / kernel load)
    last = None
    if not torch.cuda.is_available():  # host candidates (CPU tests of the selection protocol)
        best = float("inf")
        for _ in range(batches):
            t0 = time.perf_counter()
            for _ in range(reps):
                last = fn()
            best = min(best, (time.perf_counter() - t0) * 1e3 / reps)
        outs.append(_snap(last, probe))
        return best, outs
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(batches):
        s.record()
        for _ in range(reps):
            last = fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    outs.append(_snap(last, probe))
    return best, outs


# candidate-vs-default tolerance, relative to the reference's largest finite magnitude: bf16 output
# rounding and fp32 summation order stay far below it (< 0.5 %); an absolute floor would let a
# candidate that returns zeros pass wherever every entry of the reference is small (a weight gradient
# of magnitude < 0.01 passed the old ``5 % + 1e-2`` rule)
AGREE_REL = 0.03


def _agrees(outs: list, ref: list) -> bool:
    for o, r in zip(outs, ref):
        if o is None or r is None:
            continue
        if o.shape != r.shape:
            return False
        fin = torch.isfinite(r)
        if not bool(torch.isfinite(o)[fin].all()):
            return False
        if not bool(fin.any()):
            continue
        d = float((o[fin] - r[fin]).abs().max())
        mx = float(r[fin].abs().max())
        # the floor is one fp32 ulp of the reference's scale: an all-zero reference demands zeros
        if d > AGREE_REL * mx + mx * 2.0 ** -23:
            return False
    return True


def rejected() -> dict:
    """Candidates dropped for wrong output, per key (for logs / tests)."""
    return dict(_REJECTED)


def _store():
    """The rendezvous store when this process is one rank of several, else None."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() <= 1:
        return None
    return dist.distributed_c10d._get_default_store()


def _peer_decision(st, skey: str, candidates: dict) -> str | None:
    """Another rank claimed ``skey``: wait for its published choice."""
    st.wait([f"psd/autotune/d/{skey}"], datetime.timedelta(seconds=float(os.environ.get("PSD_AUTOTUNE_WAIT_S", "900"))))
    name = st.get(f"psd/autotune/d/{skey}").decode()
    if name == _DECLINED:
        raise Declined(f"autotune {skey}: every candidate declined on the deciding rank")
    if name.startswith(_FAILED):
        raise RuntimeError(f"autotune {skey}: the deciding rank failed: {name[len(_FAILED) + 1:]}")
    if name not in candidates:
        raise RuntimeError(f"autotune: rank decision {name!r} for {skey} is not a candidate here {sorted(candidates)}")
    return name


def choose(key: tuple, candidates: dict, default: str, probe=None, group=None) -> str:
    """Name of the fastest *correct* candidate for ``key`` (timed and validated once, cached).
    ``probe``: returns the output tensor of a candidate that writes into a preallocated buffer
    instead of returning its result. ``group``: name -> family, for candidate sets whose families
    return different (each internally consistent) tensors -- e.g. a fused bwd-data epilogue returns
    the BN-masked gradient, the plain kernels dX: each candidate is validated against the first
    candidate of its own family (the default's family against the default)."""
    full = candidates
    lib_fallback = {}
    if not _feat("library_linear" if key and key[0] == "linear" else "library_candidates"):
        # our kernels only: a library candidate (MIOpen / hipBLASLt) stays only where no kernel of
        # ours takes the shape -- the reference of the correctness check is then our default kernel;
        # if every one of ours declines at run time, the library candidates are timed after all
        own = {n: f for n, f in candidates.items() if n not in LIBRARY}
        if own:
            lib_fallback = {n: f for n, f in candidates.items() if n in LIBRARY}
            candidates = own
            if default not in own:
                default = next(iter(own))
    got = _DECISIONS.get(key)
    if got is not None and got in full:
        return got
    if key in _DECLINED_KEYS:
        raise Declined(f"autotune {key}: every candidate declined")
    # A/B runs: e.g. "mfma" / "blas" / "miopen" / "gemm", or a priority list "psdnb0,psdn0" (the
    # first name this op offers wins)
    for forced in os.environ.get("PSD_AUTOTUNE_FORCE", "").split(","):  # (a forced library name overrides the filter)
        if forced and forced in full:
            _DECISIONS[key] = forced
            return forced
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return default
    st = _store()
    skey = repr(key)
    if st is not None and int(st.add(f"psd/autotune/c/{skey}", 1)) > 1:
        try:
            best = _peer_decision(st, skey, full)
        except Declined:
            _DECLINED_KEYS.add(key)
            raise
        _DECISIONS[key] = best
        _SOURCE["peer"] += 1
        return best
    # The claiming rank always publishes -- a decision, "every candidate declined", or its error --
    # so no peer waits on a key nobody will decide (and this rank never claims it again).
    try:
        try:
            best = _time_and_pick(key, candidates, default, probe, group)
        except Declined:
            if not lib_fallback:
                raise
            best = _time_and_pick(key, lib_fallback, next(iter(lib_fallback)), probe, group)
    except Declined:
        _DECLINED_KEYS.add(key)
        if st is not None:
            st.set(f"psd/autotune/d/{skey}", _DECLINED)
        raise
    except BaseException as e:
        if st is not None:
            st.set(f"psd/autotune/d/{skey}", f"{_FAILED}:{type(e).__name__}: {e}"[:512])
        raise
    if st is not None:
        st.set(f"psd/autotune/d/{skey}", best)
        _SOURCE["claimed"] += 1
    else:
        _SOURCE["local"] += 1
    return best


# candidate names that run a library kernel (MIOpen, hipBLASLt through torch.mm / F.linear)
LIBRARY = frozenset({"miopen", "gemm", "blas"})
OWN_MARGIN = 0.02


def _time_and_pick(key: tuple, candidates: dict, default: str, probe, group=None) -> str:
    runs, declined = {}, []
    for name, fn in candidates.items():
        try:
            runs[name] = _time_ms(fn, probe=probe)
        except Declined:
            declined.append(name)
    if declined:
        _REJECTED[key] = [f"declined:{n}" for n in declined]
    if not runs:
        raise Declined(f"autotune {key}: every candidate declined ({declined})")
    ref_name = default if default in runs else next(iter(runs))
    ref = runs[ref_name][1]
    if any(o is not None and not bool(torch.isfinite(o).all()) for o in ref):
        # the default itself misbehaves: judge against any candidate with a finite output
        ref_name = next((n for n, r in runs.items() if all(o is None or bool(torch.isfinite(o).all())
                                                           for o in r[1])), ref_name)
        ref = runs[ref_name][1]
    if group is None:
        ok = {n: r[0] for n, r in runs.items() if n == ref_name or _agrees(r[1], ref)}
    else:
        refs = {group(ref_name): ref_name}  # per family: the default, else the family's first candidate
        for n in runs:
            refs.setdefault(group(n), n)
        ok = {n: r[0] for n, r in runs.items() if n == refs[group(n)] or _agrees(r[1], runs[refs[group(n)]][1])}
    bad = [n for n in runs if n not in ok]
    if bad:
        _REJECTED[key] = _REJECTED.get(key, []) + bad
    best = min(ok, key=ok.get)
    if best in LIBRARY and _feat("prefer_own"):
        # one of our kernels within OWN_MARGIN of a library winner takes the pick: closer than the
        # run-to-run spread of one kernel's timing, such a decision flipped the library kernel in and
        # out of the step from box to box (2-7 MIOpen weight gradients per ResNet-50 step)
        own = {n: t for n, t in ok.items() if n not in LIBRARY}
        if own:
            o = min(own, key=own.get)
            if own[o] <= ok[best] * (1.0 + OWN_MARGIN):
                best = o
    _DECISIONS[key] = best
    _TIMES[key] = {n: round(r[0], 4) for n, r in runs.items()}
    if os.environ.get("PSD_AUTOTUNE_LOG"):
        print(f"[autotune] {key}: {_TIMES[key]} -> {best}" + (f" (rejected {bad})" if bad else ""), flush=True)
    return best


def source() -> dict:
    """How this rank's decisions were made: timed here with no peers ("local"), timed here for
    every rank ("claimed"), taken from the rank that timed them ("peer"), or loaded ("file")."""
    return dict(_SOURCE)


# Decision-file schema: bump whenever a candidate's name starts to mean a different kernel (the
# psdw / convn variant numbering changed in round 5: a file from before would pin other kernels
# under the same names). Files of another schema are refused, never half-applied.
SCHEMA = "psd-autotune/6"


def save_decisions(path: str) -> None:
    """Write this process's decisions as JSON (``PSD_AUTOTUNE_FILE`` loads them)."""
    dec = {repr(k): v for k, v in sorted(_DECISIONS.items(), key=lambda kv: repr(kv[0]))}
    with open(path, "w") as f:
        json.dump({"schema": SCHEMA, "decisions": dec}, f, indent=1)


def load_decisions(path: str) -> int:
    """Pin the decisions of a ``save_decisions`` file; returns how many were loaded. A file without
    this build's ``SCHEMA`` (older variant numbering) raises ValueError."""
    with open(path) as f:
        raw = json.load(f)
    if not isinstance(raw, dict) or raw.get("schema") != SCHEMA:
        got = raw.get("schema") if isinstance(raw, dict) else None
        raise ValueError(f"autotune decision file {path}: schema {got!r}, this build reads {SCHEMA!r} "
                         "(candidate names changed meaning; re-time and save a new file)")
    for k, v in raw["decisions"].items():
        key = ast.literal_eval(k)
        _DECISIONS[key] = v
        _FILE_KEYS.add(key)
    _SOURCE["file"] = len(_FILE_KEYS)
    return len(raw["decisions"])


if os.environ.get("PSD_AUTOTUNE_FILE"):
    load_decisions(os.environ["PSD_AUTOTUNE_FILE"])


def times() -> dict:
    """ms per call of every timed candidate, per key (for logs / bench JSON)."""
    return dict(_TIMES)


def decisions() -> dict:
    return dict(_DECISIONS)


def set_decision(key: tuple, name: str | None) -> None:
    """Pin (or with ``None`` forget) the choice for ``key`` (tests)."""
    if name is None:
        _DECISIONS.pop(key, None)
    else:
        _DECISIONS[key] = name
