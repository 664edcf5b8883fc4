#!/bin/bash
# Profile N timed bench steps under rocprofv3 on the GPU box and leave only small summaries in
# gpurun_out/ (the raw trace of a ResNet-50 run is >64 MiB).  Usage: scripts/gpu_profile_bench.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run --output-format csv -- \
  python3 "$R/bench.py" "$@" --out "$OUT/bench.json" > "$OUT/run.log" 2>&1
rc=$?
T=$(find /tmp/prof_$TAG -name "*kernel_trace.csv" | head -1)
if [ -n "$T" ]; then
  python3 "$R/tools/prof_summary.py" "$T" --steps 5 --title "$TAG" > "$OUT/summary.md" 2>>"$OUT/run.log"
  gzip -c "$T" > "$OUT/kernel_trace.csv.gz"
  [ "$(stat -c %s "$OUT/kernel_trace.csv.gz")" -gt 20000000 ] && rm -f "$OUT/kernel_trace.csv.gz"
fi
exit $rc
