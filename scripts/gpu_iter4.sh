#!/bin/bash
# narrow-conv tests, tail / convh microbenches, one bench run (round-4 iteration)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/it4
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convn.py tests/test_tail.py tests/test_bnfold.py tests/test_convw.py > "$OUT/tests.txt" 2>&1
rc=$?; tail -2 "$OUT/tests.txt"
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" "$OUT/tests.txt" | head -20; exit $rc; fi
timeout -k 10 300 python3 tools/tail_bench.py > "$OUT/tail_bench.md" 2>&1 || { tail -20 "$OUT/tail_bench.md"; exit 1; }
cat "$OUT/tail_bench.md"
timeout -k 10 300 python3 tools/convh_bench.py > "$OUT/convh_bench.md" 2>&1 || { tail -20 "$OUT/convh_bench.md"; exit 1; }
grep "|" "$OUT/convh_bench.md"
PSD_AUTOTUNE_LOG=1 PSD_STEP_LOG=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'])"
grep "tail" "$OUT/bench.log" | head -20
