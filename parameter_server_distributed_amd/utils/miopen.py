"""Ship MIOpen's tuned find-db with the repo (for the library fallback).

Since round 6 the benches run no MIOpen kernel: every ResNet-50 / WRN-101-2 convolution shape is
taken by our kernels and the library is no longer an autotune candidate there (feature
``library_candidates``, utils/config.py), so the prebuilt MIOpen kernel cache (a binary
``.ukdb``) is no longer shipped. MIOpen stays the fallback for shapes none of our kernels takes
(and the fp32 reference of tests); ``tuning/miopen/db`` holds its text find-db produced on gfx950,
and ``install()`` copies it to a writable scratch directory and points MIOpen at it
(MIOPEN_USER_DB_PATH / MIOPEN_CUSTOM_CACHE_DIR), so a fallback compiles only what it uses. Must run
before the first convolution (ideally before ``import torch``).
"""
from __future__ import annotations

import atexit
import os
import shutil
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "tuning", "miopen")


def install(force: bool = False) -> str | None:
    if not force and ("MIOPEN_USER_DB_PATH" in os.environ or os.environ.get("PSD_NO_MIOPEN_DB") == "1"):
        return os.environ.get("MIOPEN_USER_DB_PATH")
    if not os.path.isdir(SRC):
        return None
    dst = os.path.join(tempfile.gettempdir(), f"psd_miopen_{os.getuid()}_{os.getpid()}")
    for sub in ("db", "cache"):
        s = os.path.join(SRC, sub)
        d = os.path.join(dst, sub)
        os.makedirs(d, exist_ok=True)
        if os.path.isdir(s):
            for f in os.listdir(s):
                shutil.copy2(os.path.join(s, f), os.path.join(d, f))
    os.environ["MIOPEN_USER_DB_PATH"] = os.path.join(dst, "db")
    os.environ["MIOPEN_CUSTOM_CACHE_DIR"] = os.path.join(dst, "cache")
    out = os.environ.get("PSD_MIOPEN_DB_OUT")
    if out:  # tuning run: export the grown database for tuning/miopen
        atexit.register(lambda: shutil.copytree(dst, out, dirs_exist_ok=True))
    return dst
