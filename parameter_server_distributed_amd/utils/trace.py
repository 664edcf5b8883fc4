"""Per-iteration phase tracing: HIP-event timers + roctx ranges, one JSON line per step per rank.

The reference had no timers or trace spans at all. ``StepTracer`` times named
phases on the compute stream (forward / backward / finish) and, through ``comm_span``, the PS
push/apply/pull work of every bucket on the comm stream; ranges also show up in rocprofv3
``--marker-trace`` via roctx (torch.cuda.nvtx maps to roctx on ROCm). Timings are resolved one step
late (events are queried, never synchronized, inside the step).
"""
from __future__ import annotations

import contextlib
import json
import os
import time

import torch


class StepTracer:
    def __init__(self, path: str | None = None, rank: int = 0, device=None):
        self.rank = rank
        self.device = device
        self.path = path
        self.f = open(path, "a") if path else None
        self.on_gpu = device is not None and torch.cuda.is_available() and torch.device(device).type == "cuda"
        self._cur: dict = {}
        self._pending: list = []
        self.records: list = []
        self._t0 = time.perf_counter()

    def _event(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.on_gpu:
            torch.cuda.nvtx.range_push(name)
            s = self._event()
            try:
                yield
            finally:
                e = self._event()
                torch.cuda.nvtx.range_pop()
                self._cur.setdefault(name, []).append((s, e))
        else:
            t = time.perf_counter()
            try:
                yield
            finally:
                self._cur.setdefault(name, []).append(time.perf_counter() - t)

    def comm_span(self, stream=None):
        """Context manager timing work enqueued on ``stream`` (the PS comm stream)."""
        if not self.on_gpu:
            return self.phase("comm")

        @contextlib.contextmanager
        def _span():
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record(stream)
            try:
                yield
            finally:
                e.record(stream)
                self._cur.setdefault("comm", []).append((s, e))

        return _span()

    def end_step(self, step: int, **extra):
        self._pending.append((step, self._cur, extra, time.perf_counter() - self._t0))
        self._cur = {}
        self._flush(block=False)

    def _flush(self, block: bool):
        keep = []
        for step, phases, extra, wall in self._pending:
            ready = True
            if self.on_gpu and not block:
                ready = all(e.query() for spans in phases.values() for v in spans if isinstance(v, tuple) for e in v)
            if not ready:
                keep.append((step, phases, extra, wall))
                continue
            rec = {"step": step, "rank": self.rank, "wall_s": round(wall, 6)}
            for name, spans in phases.items():
                ms = 0.0
                for v in spans:
                    if isinstance(v, tuple):
                        v[1].synchronize()
                        ms += v[0].elapsed_time(v[1])
                    else:
                        ms += v * 1e3
                rec[f"{name}_ms"] = round(ms, 4)
            rec.update(extra)
            self.records.append(rec)
            if self.f:
                self.f.write(json.dumps(rec) + "\n")
        self._pending = keep

    def close(self):
        self._flush(block=True)
        if self.f:
            self.f.close()
            self.f = None


def rank_path(path: str, rank: int) -> str:
    root, ext = os.path.splitext(path)
    return f"{root}.rank{rank}{ext or '.jsonl'}"
