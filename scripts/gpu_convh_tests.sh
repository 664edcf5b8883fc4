#!/bin/bash
# narrow-conv GPU tests, then the convh microbench with kernel stats (gpurun_out/convh/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/convh
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_convn.py tests/test_convw.py tests/test_bn.py tests/test_bnfold.py tests/test_tail.py \
  > "$OUT/tests.txt" 2>&1 || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ch -o run --output-format csv -- python3 "$R/tools/convh_bench.py" \
  > "$OUT/bench.md" 2>&1 || { tail -30 "$OUT/bench.md"; exit 1; }
grep "|\|rel" "$OUT/bench.md"
f=$(find /tmp/ch -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kstats.csv"
echo done
