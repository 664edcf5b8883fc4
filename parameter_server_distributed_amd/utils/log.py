"""Structured logging with role/rank prefixes (the reference only had bare std::cout lines)."""
from __future__ import annotations

import logging
import os
import sys

_FMT = "%(asctime)s.%(msecs)03d %(levelname).1s [%(name)s%(rank)s] %(message)s"


class _RankFilter(logging.Filter):
    def filter(self, record):
        r = os.environ.get("RANK")
        record.rank = f"/r{r}" if r is not None else ""
        return True


def get_logger(role: str) -> logging.Logger:
    lg = logging.getLogger(f"psd.{role}")
    if not lg.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter(_FMT, datefmt="%H:%M:%S"))
        h.addFilter(_RankFilter())
        lg.addHandler(h)
        lg.setLevel(os.environ.get("PSD_LOG_LEVEL", "INFO").upper())
        lg.propagate = False
    return lg
