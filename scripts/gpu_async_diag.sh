#!/bin/bash
# async-plane step timing: per-step host times of the timed loop at 10 and 30 steps, and sync S=0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/adiag
mkdir -p "$OUT"
cd "$R"
for cfg in "--steps 30 --warmup 5" "--steps 10 --warmup 5" "--steps 30 --warmup 5 --staleness 0"; do
  tag=$(echo $cfg | tr -d ' -')
  PSD_STEP_LOG=1 timeout -k 10 300 python3 bench.py $cfg --out "$OUT/$tag.json" > "$OUT/$tag.log" 2>&1 || { tail -20 "$OUT/$tag.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));print('$cfg:', d['value'], d['ms_per_step'], d['staleness_hist'])"
  grep "step host ms" "$OUT/$tag.log"
done
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_tail.py -k resnet > "$OUT/test.txt" 2>&1
grep -E "^E  .*Error|passed|failed" "$OUT/test.txt" | cut -c1-3000
exit 0
