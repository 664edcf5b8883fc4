#!/bin/bash
# BERT-side GPU tests, then a rocprofv3 breakdown of BERT-base b256 and a plain BERT bench. Usage: scripts/gpu_bert_check.sh TAG
set -o pipefail
TAG=${1:-b}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_layernorm.py tests/test_attention.py tests/test_gemm.py tests/test_fp8_training.py tests/test_kernels.py -m gpu -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
echo "tests rc=$?" >> "$OUT/gpu_tests.txt"
tail -3 "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bench_bert.json" > "$OUT/bench_bert.log" 2>&1 || exit $?
bash scripts/gpu_profile_bench.sh ${TAG}_bert --model bert_base --steps 10 --warmup 5
