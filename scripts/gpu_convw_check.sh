#!/bin/bash
# convw tests + microbench, then a rocprofv3 kernel-trace of the microbench (kernel vs reduce split).
# Usage: scripts/gpu_convw_check.sh TAG
set -o pipefail
TAG=${1:-cw}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 200 python -u -m pytest tests/test_convw.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
timeout -k 10 300 python tools/convw_bench.py > "$OUT/bench.md" 2>&1 || { cat "$OUT/bench.md"; exit 1; }
cat "$OUT/bench.md"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/cwprof -o run --output-format csv -- python3 "$R/tools/convw_bench.py" --reps 3 > "$OUT/prof.log" 2>&1 || exit $?
f=$(find /tmp/cwprof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv"
exit 0
