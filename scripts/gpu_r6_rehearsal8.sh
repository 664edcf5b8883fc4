#!/bin/bash
# the driver's N = 8 path rehearsed on ONE MI355X (8 ranks sharing the GPU over
# gloo + real IPC), three BASELINE configs at small batch, each JSON checked by
# tools/rehearsal_check.py; then the scatter kernel's cost to a concurrent backward
# (tools/xfer_interference.py). Usage: scripts/gpu_r6_rehearsal8.sh TAG
set -o pipefail
TAG=${1:-rh8}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
run8() {  # name port bench-args...
  local name=$1 port=$2; shift 2
  timeout -k 10 420 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port "$port" bench.py --gpus 8 --backend gloo --steps 4 --warmup 2 --out "$OUT/$name.json" "$@" \
    > "$OUT/$name.log" 2>&1 || { echo "$name rc=$?"; tail -20 "$OUT/$name.log"; return 1; }
  python3 tools/rehearsal_check.py "$OUT/$name.json" --world 8 | tee "$OUT/$name.check.txt"
}
run8 config3_resnet50 29711 --model resnet50 --batch 32 --ps-shards 2 --staleness 1 || exit 1
run8 config4_bert 29712 --model bert_base --batch 16 --placement disjoint --optimizer adamw --staleness 1 || exit 1
run8 config5_wrn 29713 --model wide_resnet101_2 --batch 8 --ps-shards 8 --staleness 1 || exit 1
timeout -k 10 300 python3 tools/xfer_interference.py --batch 256 --owners 2 --json "$OUT/xfer_interference.json" \
  > "$OUT/xfer_interference.md" 2>&1
