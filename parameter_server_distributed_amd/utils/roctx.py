"""rocprofv3 collection window from inside the program: ``roctxProfilerPause`` / ``Resume`` of the
ROCm profiler SDK's roctx library, which ``rocprofv3 --selected-regions`` honours (only what runs
between a resume and the next pause is traced; collection starts paused, and a pause before the
first resume aborts the tool). bench.py ``--prof-window`` resumes for the timed steps only, so a trace or counter pass holds the steps of interest and not
the start-up autotune (whose API calls alone overflow a 64 MiB result budget)."""
from __future__ import annotations

import ctypes

_lib = None


def _roctx():
    global _lib
    if _lib is None:
        try:
            _lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
        except OSError:
            _lib = False
    return _lib or None


def pause() -> bool:
    lib = _roctx()
    if lib is None:
        return False
    lib.roctxProfilerPause(ctypes.c_uint64(0))
    return True


def resume() -> bool:
    lib = _roctx()
    if lib is None:
        return False
    lib.roctxProfilerResume(ctypes.c_uint64(0))
    return True
