#!/bin/bash
# attention GPU tests + BERT bench, then a rocprofv3 breakdown of WRN-101-2 (fp8 compute)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/s2d
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_attention.py tests/test_layernorm.py tests/test_conv_igemm.py tests/test_gemm.py -m gpu -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bench_bert.json" > "$OUT/bench_bert.log" 2>&1 || exit $?
bash scripts/gpu_profile_bench.sh s2d_wrn --model wide_resnet101_2 --steps 8 --warmup 4 || exit $?
timeout -k 10 400 python3 bench.py --model wide_resnet101_2 --steps 10 --warmup 4 --out "$OUT/bench_wrn.json" > "$OUT/bench_wrn.log" 2>&1
