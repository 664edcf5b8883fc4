"""``parameter_server [listen_addr] [total_workers] [checkpoint_interval] [--flags]`` -- argv-compatible
with the reference's parameter_main (src/parameter_main.cpp:5-22: defaults 0.0.0.0:50051, 2, 10)."""
from __future__ import annotations

import argparse

from ..ops.optim import OptimConfig
from ..runtime.parameter_server import serve


def main(argv=None):
    ap = argparse.ArgumentParser(prog="parameter_server")
    ap.add_argument("listen", nargs="?", default="0.0.0.0:50051")
    ap.add_argument("total_workers", nargs="?", type=int, default=2)
    ap.add_argument("checkpoint_interval", nargs="?", type=int, default=10)
    ap.add_argument("--device", default="cpu", help="cpu (host memory, like the reference) or cuda[:i] (HBM shard)")
    ap.add_argument("--mode", default="sync", choices=["sync", "async"])
    ap.add_argument("--staleness", type=int, default=-1, help="async SSP bound S (-1: unbounded)")
    ap.add_argument("--staleness-lr-scaling", action="store_true", help="async: lr / (1 + staleness)")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "momentum", "adam", "adamw"])
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weight-decay", type=float, default=0.0)
    ap.add_argument("--reference-compat", action="store_true",
                    help="reference semantics: first aggregate becomes the params, p -= g (lr 1)")
    ap.add_argument("--coordinator", default="", help="follow live membership from this coordinator")
    ap.add_argument("--ckpt-dir", default=".")
    ap.add_argument("--resume-latest", action="store_true",
                    help="load the newest checkpoint_epoch_<N>.ckpt in --ckpt-dir at start (supervised restarts)")
    from ..utils.config import apply_config

    apply_config(ap, argv)
    a = ap.parse_intermixed_args(argv)
    opt = OptimConfig(a.optimizer, lr=a.lr, momentum=a.momentum if a.optimizer == "momentum" else 0.0,
                      weight_decay=a.weight_decay)
    serve(a.listen, a.total_workers, a.checkpoint_interval, device=a.device, optim=opt, mode=a.mode,
          staleness=a.staleness, reference_compat=a.reference_compat, ckpt_dir=a.ckpt_dir,
          coordinator=a.coordinator or None, staleness_lr_scaling=a.staleness_lr_scaling,
          resume_latest=a.resume_latest)


if __name__ == "__main__":
    main()
