#!/bin/bash
# tail test (fp32-referenced), then a same-box A/B of the recomputing tail, then the sync-SGD row.
# A test FAILURE (exit 1) does not stop the benches; a timeout / crash (any other status) does.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/tailab
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_tail.py -k resnet > "$OUT/test.txt" 2>&1
rc=$?
grep -E "^E  .*Error|passed|failed" "$OUT/test.txt" | cut -c1-6000
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "test run ended with $rc: stopping"; exit $rc; fi
bash scripts/gpu_ab.sh tail "PSD_TAIL_RECOMPUTE=0" "PSD_TAIL_RECOMPUTE=1" || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --staleness 0 --out "$OUT/sync.json" > "$OUT/sync.log" 2>&1 || { tail -20 "$OUT/sync.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/sync.json'));print('sync S=0:', d['value'], d['ms_per_step'], d['final_loss'], d.get('staleness_p50'))"
PSD_TAIL_RECOMPUTE=1 PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh r4tail --steps 10 --warmup 5 || exit $?
head -45 "$R/gpurun_out/prof_r4tail/summary.md"
