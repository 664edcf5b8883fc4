#!/bin/bash
# Round-6 call A: the new async GPU tests (self-test fallback, xfer with the release fence), then the
# 8-rank rehearsal on one GPU (scripts/gpu_r6_rehearsal8.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/r6a
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_async_ps.py -m gpu -x -v --timeout 180 --timeout-method thread \
  -k "selftest or xfer_kernel or ipc_matches" > "$OUT/async_tests.txt" 2>&1
rc=$?; tail -5 "$OUT/async_tests.txt"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r6_rehearsal8.sh r6a_rh8
