#!/usr/bin/env python3
"""Assertions on a multi-rank bench.py JSON (the N > 1 rehearsal):

* the async peer-memory plane ran (no fallback to the collective plane) on the scatter / gather
  kernels (``async_xfer == "kernel"``, no transport fallback);
* every autotune decision came through the rendezvous store: one rank timed each key ("claimed"),
  the others took its choice ("peer"), none timed alone ("local") or read a file;
* the staleness histogram holds exactly one entry per (worker push, shard): W x (warmup + steps) x P,
  all within the SSP bound;
* the weights and the loss are finite.

  python tools/rehearsal_check.py BENCH.json --world 8      (exit 1 on any failure)
"""
import argparse
import json
import sys


def check(rec: dict, world: int) -> list[str]:
    bad = []
    cfg = rec.get("config", {})
    if rec.get("n_gpus") != world:
        bad.append(f"n_gpus {rec.get('n_gpus')} != world {world}")
    if cfg.get("ps_mode") != "async" or cfg.get("async_fallback"):
        bad.append(f"async plane fell back: ps_mode={cfg.get('ps_mode')} fallback={cfg.get('async_fallback')}")
    if cfg.get("async_xfer") != "kernel" or cfg.get("async_xfer_fallback"):
        bad.append(f"transport: async_xfer={cfg.get('async_xfer')} fallback={cfg.get('async_xfer_fallback')}")
    src = rec.get("autotune_source", {})
    if src.get("local", 0) or src.get("file", 0) or not src.get("claimed", 0):
        bad.append(f"autotune_source {src}: expected only claimed / peer decisions")
    W = len(cfg.get("worker_ranks", []))
    P = cfg.get("ps_shards", 0)
    want = W * (rec.get("steps", 0) + rec.get("warmup", 0)) * P
    hist = rec.get("staleness_hist") or []
    if sum(hist) != want:
        bad.append(f"staleness histogram total {sum(hist)} != W {W} x steps {rec.get('steps')}+{rec.get('warmup')} "
                   f"x shards {P} = {want}")
    S = cfg.get("staleness_bound", 0)
    # a push may be up to S + 1 steps stale (bench.py ps_semantics)
    if any(c for i, c in enumerate(hist) if i > S + 1):
        bad.append(f"staleness beyond the bound {S}: {hist}")
    if not rec.get("params_finite"):
        bad.append("non-finite weights or loss")
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("json")
    ap.add_argument("--world", type=int, required=True)
    a = ap.parse_args()
    with open(a.json) as f:
        rec = json.loads(f.read().strip().splitlines()[-1])
    bad = check(rec, a.world)
    cfg = rec.get("config", {})
    print(f"{a.json}: {rec.get('metric')} {rec.get('value')} ({cfg.get('parallelism')}), "
          f"xfer={cfg.get('async_xfer')} blocks={rec.get('async_xfer_blocks')} bucket={rec.get('bucket_mb_chosen')} MB, "
          f"autotune={rec.get('autotune_source')} hist={rec.get('staleness_hist')}")
    for b in bad:
        print("FAIL:", b)
    print("OK" if not bad else f"{len(bad)} failure(s)")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
