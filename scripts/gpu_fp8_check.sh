#!/bin/bash
# fp8 kernel tests + WRN-101-2 fp8 bench and profile
set -o pipefail
TAG=${1:-f8}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${TAG}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_kernels.py tests/test_conv_igemm.py tests/test_gemm.py -m gpu -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --model wide_resnet101_2 --steps 10 --warmup 4 --out "$OUT/bench_wrn.json" > "$OUT/bench_wrn.log" 2>&1 || exit $?
bash scripts/gpu_profile_bench.sh ${TAG}_wrn --model wide_resnet101_2 --steps 8 --warmup 4
