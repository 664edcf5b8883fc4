#!/bin/bash
# round 5: the recomputing tail's statistics (fp32 moments, fp32 apply) -- probe, then the tail /
# bnfold / bn tests three times (three consecutive passing runs). Usage: TAG
set -o pipefail
TAG=${1:-tail}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u tools/probes/tail_stats_probe.py > "$OUT/probe.txt" 2>&1 || { tail -30 "$OUT/probe.txt"; exit 1; }
grep -E "^loss|worst" "$OUT/probe.txt"
for i in 1 2 3; do
  timeout -k 10 500 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_tail.py tests/test_bnfold.py > "$OUT/tests$i.txt" 2>&1 || { grep -E "Error|assert|FAILED|^E " "$OUT/tests$i.txt" | head -30; exit 1; }
  grep -E "passed|loss fp32" "$OUT/tests$i.txt"
done
