#!/bin/bash
# tail / BN / fold tests + the 1-GPU bench (default flags), after a change to the tail or BN paths
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-small}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_tail.py tests/test_bnfold.py tests/test_bn.py -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
timeout -k 10 400 python -u bench.py --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['final_loss'],d['params_finite'])"
