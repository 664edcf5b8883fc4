"""``coordinator [listen_addr] [ps_host[:port]] [--flags]`` -- argv-compatible with the reference's
coordinator_main (src/coordinator_main.cpp:5-24: defaults 0.0.0.0:50052 and localhost:50051)."""
from __future__ import annotations

import argparse

from ..runtime.coordinator import serve


def main(argv=None):
    ap = argparse.ArgumentParser(prog="coordinator")
    ap.add_argument("listen", nargs="?", default="0.0.0.0:50052")
    ap.add_argument("ps_address", nargs="?", default="localhost:50051")
    ap.add_argument("--expiry-s", type=float, default=30.0, help="drop workers silent for longer (reference: 30)")
    ap.add_argument("--sweep-s", type=float, default=10.0, help="expiry sweep period (reference: 10)")
    ap.add_argument("--shards", default="", help="comma-separated PS shard addresses (default: the PS address)")
    ap.add_argument("--store-port", type=int, default=0,
                    help="rendezvous store port for elastic collective workers (0: any free port, -1: none)")
    from ..utils.config import apply_config

    apply_config(ap, argv)
    a = ap.parse_intermixed_args(argv)
    shards = [s for s in a.shards.split(",") if s]
    serve(a.listen, a.ps_address, a.expiry_s, a.sweep_s, shards,
          store_port=None if a.store_port < 0 else a.store_port)


if __name__ == "__main__":
    main()
