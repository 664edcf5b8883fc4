#!/bin/bash
# GEMM numerics (tests/test_gemm.py) then the timing tables of tools/gemm_probe.py.
# Usage: scripts/gpu_gemm_check.sh TAG [extra probe args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/gemmcheck_$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gemm.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -3 "$OUT/tests.txt"
timeout -k 10 300 python3 tools/gemm_probe.py --shapes all "$@" > "$OUT/table.md" 2> "$OUT/table.err" || exit $?
timeout -k 10 200 python3 tools/gemm_probe.py --ksweep NTx32768x3072 > "$OUT/ksweep_nt.md" 2>> "$OUT/table.err" || exit $?
cat "$OUT/table.md" "$OUT/ksweep_nt.md"
