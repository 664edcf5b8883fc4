#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/lnbias
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_layernorm.py tests/test_gemm.py -k "layernorm or bias or gelu or linear or handoff or dropout" > "$OUT/tests.txt" 2>&1
rc=$?; tail -2 "$OUT/tests.txt"
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" "$OUT/tests.txt" | head -20; exit $rc; fi
timeout -k 10 400 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bert.json" > "$OUT/bert.log" 2>&1 || { tail -20 "$OUT/bert.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bert.json'));print('bert', d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'])"
