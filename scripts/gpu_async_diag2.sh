#!/bin/bash
# async S=1 with / without the persistent kernels (do they lose CUs to the PS apply running beside them?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/adiag2
mkdir -p "$OUT"
cd "$R"
run() {
  tag=$1; shift
  env "$@" PSD_STEP_LOG=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/$tag.json" > "$OUT/$tag.log" 2>&1 || { tail -20 "$OUT/$tag.log"; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['staleness_hist'])"
  grep "step host ms" "$OUT/$tag.log" | cut -c1-200
}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convn.py tests/test_tail.py tests/test_bnfold.py > "$OUT/tests.txt" 2>&1
rc=$?
tail -3 "$OUT/tests.txt"
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED|Error" "$OUT/tests.txt" | head -20; exit $rc; fi
run async_default PSD_X=1 || exit 1
run async_nopersist PSD_CONVN_PERSIST=0 PSD_CONVW_PERSIST=0 PSD_CONVN_P1=0 || exit 1
run async_nop1 PSD_CONVN_P1=0 || exit 1
run async_tail PSD_TAIL_RECOMPUTE=1 || exit 1
exit 0
