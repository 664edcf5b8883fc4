#!/bin/bash
# Round-6 baseline: plain ResNet-50 bench, BERT bench with the autotune log, and a BERT rocprof table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/r6base
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/bench_r50.json" > "$OUT/bench_r50.log" 2>&1 || exit $?
PSD_AUTOTUNE_LOG=1 timeout -k 10 300 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bench_bert.json" > "$OUT/bench_bert.log" 2>&1 || exit $?
PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh r6base_bert --model bert_base --steps 10 --warmup 5
