#!/bin/bash
# end-of-round-4 check: dual-tail nobx tests + A/B, then the full GPU suite + rocprof bench + rehearsal
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/final4
mkdir -p "$OUT"
cd "$R"
PSD_DUAL_NOBX=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bnfold.py tests/test_bn.py tests/test_tail.py > "$OUT/nobx_tests.txt" 2>&1
rc=$?; tail -1 "$OUT/nobx_tests.txt"
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" "$OUT/nobx_tests.txt" | head -20; exit $rc; fi
bash scripts/gpu_ab_env.sh PSD_DUAL_NOBX "1 0 1 0" || exit $?
bash scripts/gpu_full_iter.sh full5 || exit $?
bash scripts/gpu_rehearsal.sh rh5 || exit $?
for f in gpurun_out/rh5/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'], d.get('final_loss'), d.get('params_finite'))"; done
