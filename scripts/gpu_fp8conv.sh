#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/fp8conv
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_fp8_training.py -k 300_step > "$OUT/tests.txt" 2>&1
rc=$?; grep -E "bf16:|passed|failed" "$OUT/tests.txt"; [ $rc -ne 0 ] && grep -E "^E  " "$OUT/tests.txt" | head; exit $rc
