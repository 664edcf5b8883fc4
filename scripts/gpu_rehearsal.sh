#!/bin/bash
# Multi-rank rehearsal on the one GPU: 2 ranks (gloo store + IPC on one device), async and collective
# planes, ResNet-50 b256 per rank. Usage: scripts/gpu_rehearsal.sh TAG
set -o pipefail
TAG=${1:-rh}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 \
  bench.py --gpus 2 --backend gloo --batch 256 --steps 10 --warmup 3 --out "$OUT/async_2rank.json" > "$OUT/async_2rank.log" 2>&1 || exit $?
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29656 \
  bench.py --gpus 2 --backend gloo --batch 256 --steps 10 --warmup 3 --ps-mode collective --out "$OUT/coll_2rank.json" > "$OUT/coll_2rank.log" 2>&1
