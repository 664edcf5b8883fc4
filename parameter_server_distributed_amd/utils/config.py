"""Run-config files (YAML or JSON) for the bench and the role CLIs.

``--config run.yaml`` supplies defaults for any long option of the command (keys use either
``ps-shards`` or ``ps_shards`` spelling); explicit command-line flags still win. Files are read
with ``yaml.safe_load`` / ``json.load`` only. The reference configures everything through
positional argv and shell-script env vars (scripts/*.sh); this is additive.
"""
from __future__ import annotations

import argparse
import json
import os


def load_config(path: str) -> dict:
    with open(path) as f:
        text = f.read()
    if path.endswith(".json"):
        cfg = json.loads(text)
    else:
        import yaml

        cfg = yaml.safe_load(text) or {}
    if not isinstance(cfg, dict):
        raise ValueError(f"{path}: a run config must be a mapping of option -> value")
    return {str(k).replace("-", "_"): v for k, v in cfg.items()}


def apply_config(ap: argparse.ArgumentParser, argv: list[str] | None = None) -> None:
    """Pre-parse ``--config`` from ``argv`` and install the file's values as parser defaults."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--config", default=os.environ.get("PSD_CONFIG", ""))
    known, _ = pre.parse_known_args(argv)
    if not any(a.dest == "config" for a in ap._actions):
        ap.add_argument("--config", default="", help="YAML/JSON run config (flags override it)")
    if not known.config:
        return
    cfg = load_config(known.config)
    dests = {a.dest for a in ap._actions}
    unknown = sorted(set(cfg) - dests)
    if unknown:
        raise SystemExit(f"{known.config}: unknown option(s) {unknown}")
    ap.set_defaults(**cfg)
