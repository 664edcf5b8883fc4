#!/bin/bash
# GPU checks for the async data plane: GPU tests, 1-GPU bench in both PS modes, 2-rank rehearsal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-r2b}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
echo "tests rc=$?" | tee -a "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/bench_async.json" > "$OUT/bench_async.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --ps-mode collective --out "$OUT/bench_coll.json" > "$OUT/bench_coll.log" 2>&1 || exit $?
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 \
  bench.py --gpus 2 --backend gloo --batch 256 --steps 10 --warmup 3 --out "$OUT/bench_async_2rank.json" > "$OUT/bench_async_2rank.log" 2>&1
exit $?
