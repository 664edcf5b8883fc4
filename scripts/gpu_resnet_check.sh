#!/bin/bash
# Full GPU test suite, then a ResNet-50 b1024 bench and a rocprofv3 breakdown. Usage: scripts/gpu_resnet_check.sh TAG
set -o pipefail
TAG=${1:-rn}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
echo "tests rc=$?" >> "$OUT/gpu_tests.txt"
tail -3 "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/bench_resnet.json" > "$OUT/bench_resnet.log" 2>&1 || exit $?
bash scripts/gpu_profile_bench.sh ${TAG}_resnet50 --steps 10 --warmup 5
