#!/bin/bash
# Session check: implicit-GEMM conv tests first, the full GPU suite, then the three benchmark models
# (ResNet-50 with a rocprofv3 breakdown, BERT-base, Wide-ResNet-101-2 fp8). Usage: scripts/gpu_all_check.sh TAG
set -o pipefail
TAG=${1:-all}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 200 python -u -m pytest tests/test_conv_igemm.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/conv_tests.txt" 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
echo "tests rc=$?" >> "$OUT/gpu_tests.txt"
tail -3 "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/bench_resnet.json" > "$OUT/bench_resnet.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bench_bert.json" > "$OUT/bench_bert.log" 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --model wide_resnet101_2 --steps 10 --warmup 4 --out "$OUT/bench_wrn.json" > "$OUT/bench_wrn.log" 2>&1 || exit $?
bash scripts/gpu_profile_bench.sh ${TAG}_resnet50 --steps 10 --warmup 5
