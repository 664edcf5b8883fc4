#!/bin/bash
# One GPU call: the GPU test suite, then rocprofv3 kernel breakdowns of the three benchmark models
# (ResNet-50 b1024, BERT-base b256, Wide-ResNet-101-2 fp8). Usage: scripts/gpu_session_check.sh TAG
set -o pipefail
TAG=${1:-s}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
echo "tests rc=$?" >> "$OUT/gpu_tests.txt"
tail -3 "$OUT/gpu_tests.txt"
bash scripts/gpu_profile_bench.sh ${TAG}_resnet50 --steps 10 --warmup 5 || exit $?
bash scripts/gpu_profile_bench.sh ${TAG}_bert --model bert_base --steps 10 --warmup 5 || exit $?
timeout -k 10 400 python3 bench.py --model wide_resnet101_2 --steps 10 --warmup 5 --out "$OUT/bench_wrn.json" > "$OUT/bench_wrn.log" 2>&1
exit $?
