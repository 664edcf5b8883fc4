#!/bin/bash
# Round-6 call B: the 192 x 256 transposed-store GEMM (gemm_ct_): GEMM tests, the BERT-shape probe
# (ours NT / CT vs hipBLASLt), then the BERT bench with the autotune log and its rocprof table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/r6b
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gemm.py -m gpu -x -q --timeout 180 --timeout-method thread \
  > "$OUT/gemm_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gemm_tests.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/gemm_probe.py --shapes bert > "$OUT/gemm_probe_bert.md" 2>&1 || exit $?
cat "$OUT/gemm_probe_bert.md"
PSD_AUTOTUNE_LOG=1 timeout -k 10 300 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bench_bert.json" \
  > "$OUT/bench_bert.log" 2>&1 || exit $?
grep autotune "$OUT/bench_bert.log" | grep "linear', '\(fwd\|dgrad\)'"
PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh r6b_bert --model bert_base --steps 10 --warmup 5
