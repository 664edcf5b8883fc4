"""``worker_main [coordinator] [worker_id] [iterations] [worker_addr] [worker_port] [checkpoint_path]``
-- argv-compatible with the reference's worker_main (src/worker_main.cpp:5-45), printing the same
``worker <id> iter <it> done=<bool>`` lines. A checkpoint path resumes from the checkpoint's
iteration (the reference restarted at 0, D11)."""
from __future__ import annotations

import argparse
import json
import signal
import sys
import time

from ..runtime.worker import Worker


def main(argv=None):
    ap = argparse.ArgumentParser(prog="worker_main")
    ap.add_argument("coordinator", nargs="?", default="localhost:50052")
    ap.add_argument("worker_id", nargs="?", type=int, default=0)
    ap.add_argument("iterations", nargs="?", type=int, default=1)
    ap.add_argument("worker_addr", nargs="?", default="")
    ap.add_argument("worker_port", nargs="?", type=int, default=0)
    ap.add_argument("checkpoint_path", nargs="?", default="")
    ap.add_argument("--model", default="mlp")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--mode", default="sync", choices=["sync", "async"])
    ap.add_argument("--heartbeat-s", type=float, default=5.0)
    ap.add_argument("--bf16-wire", action="store_true", help="push gradients as bf16 bytes")
    ap.add_argument("--reference-wire", action="store_true",
                    help="encode tensors as the reference did (repeated float), not bulk bytes")
    ap.add_argument("--stats-json", default="", help="write final PS stats + losses to this file")
    from ..utils.config import apply_config

    apply_config(ap, argv)
    a = ap.parse_intermixed_args(argv)
    w = Worker(a.coordinator, a.worker_id, a.worker_addr, a.worker_port, model=a.model, batch=a.batch,
               device=a.device, heartbeat_s=a.heartbeat_s, bf16_wire=a.bf16_wire, mode=a.mode,
               raw_wire=not a.reference_wire)
    w.initialize()

    def _leave(signum, frame):  # scale_workers.sh down: deregister so the barrier shrinks at once
        print(f"worker {a.worker_id} leaving (signal {signum})", flush=True)
        w.shutdown(deregister=True)
        sys.exit(0)

    signal.signal(signal.SIGTERM, _leave)
    start = w.start_iteration
    if a.checkpoint_path:
        epoch, it = w.load_checkpoint_from_server(a.checkpoint_path)
        start = it + 1 if it > 0 else 0
        print(f"worker {a.worker_id} loaded checkpoint epoch {epoch}, resuming at iteration {start}", flush=True)
    losses, iter_s = [], []
    t0 = time.time()
    ok_all = True
    for it in range(start, start + a.iterations):
        ti = time.time()
        done, loss, r = w.run_iteration(it)
        iter_s.append(time.time() - ti)
        losses.append(loss)
        ok_all &= done
        print(f"worker {a.worker_id} iter {it} done={'true' if done else 'false'} loss={loss:.4f} "
              f"version={r.version} staleness={r.staleness}", flush=True)
    dt = time.time() - t0
    print(f"worker {a.worker_id} finished {a.iterations} iterations in {dt:.2f} s "
          f"({a.iterations / max(dt, 1e-9):.1f} it/s)", flush=True)
    if a.stats_json:
        st = w.stats()
        with open(a.stats_json, "w") as f:
            json.dump({"losses": losses, "iter_seconds": iter_s, "version": st.version,
                       "hist": list(st.staleness_histogram),
                       "counters": json.loads(st.counters_json or "{}"), "seconds": dt}, f)
    w.shutdown()
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
