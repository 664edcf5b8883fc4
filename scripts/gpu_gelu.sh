#!/bin/bash
# GELU-backward GEMM epilogue: GEMM tests, then a same-box BERT A/B of PSD_GELU_FUSE
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/gelu
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm.py -k "gelu" > "$OUT/tests.txt" 2>&1
rc=$?; tail -2 "$OUT/tests.txt"
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" "$OUT/tests.txt" | head -20; exit $rc; fi
for v in 1 0; do
  PSD_GELU_FUSE=$v PSD_AUTOTUNE_LOG=1 timeout -k 10 400 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bert$v.json" > "$OUT/bert$v.log" 2>&1 || { tail -20 "$OUT/bert$v.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bert$v.json'));print('bert fuse=$v', d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'])"
done
grep "dgrad_gelu" "$OUT/bert1.log" | head -3
