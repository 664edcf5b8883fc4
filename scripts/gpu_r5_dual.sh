#!/bin/bash
# round 5: the recomputing dual tail -- tail / bnfold / stream-census tests, then a same-box A/B
set -o pipefail
TAG=${1:-dual}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_tail.py tests/test_bnfold.py tests/test_stream_census.py > "$OUT/tests.txt" 2>&1 || { grep -E "Error|assert|FAILED|^E " "$OUT/tests.txt" | head -30; exit 1; }
grep -E "passed|loss fp32|streams, GPU" "$OUT/tests.txt"
bash scripts/gpu_ab_env.sh dual_recompute "1 0 1 0" || exit $?
