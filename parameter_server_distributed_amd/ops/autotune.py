"""Per-shape choice between implementations of one op, timed once with HIP events.

The role MIOpen's Find plays for convolutions, for the places where this framework has both a
hand-written gfx950 kernel and a library path (hipBLASLt / MIOpen) for the same math: the first
eager call of a shape times every candidate (one warm call + 3 timed), caches the fastest and
uses it from then on. Inside a hipGraph capture nothing is timed: an undecided shape takes the
``default`` candidate (the Trainer always runs eager warmup steps before it captures).
"""
from __future__ import annotations

import os

import torch

_DECISIONS: dict[tuple, str] = {}


def enabled(var: str) -> bool:
    return os.environ.get(var, "1") != "0"


def _time_ms(fn, reps: int = 3) -> float:
    fn()  # warm (library heuristics / kernel load)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def choose(key: tuple, candidates: dict, default: str) -> str:
    """Name of the fastest candidate for ``key`` (timed once, cached)."""
    got = _DECISIONS.get(key)
    if got is not None:
        return got
    forced = os.environ.get("PSD_AUTOTUNE_FORCE")  # e.g. "mfma" / "blas" / "miopen" / "gemm": A/B runs
    if forced and forced in candidates:
        _DECISIONS[key] = forced
        return forced
    if torch.cuda.is_current_stream_capturing():
        return default
    times = {name: _time_ms(fn) for name, fn in candidates.items()}
    best = min(times, key=times.get)
    _DECISIONS[key] = best
    return best


def decisions() -> dict:
    return dict(_DECISIONS)


def set_decision(key: tuple, name: str | None) -> None:
    """Pin (or with ``None`` forget) the choice for ``key`` (tests)."""
    if name is None:
        _DECISIONS.pop(key, None)
    else:
        _DECISIONS[key] = name
