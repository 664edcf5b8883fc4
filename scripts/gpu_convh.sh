#!/bin/bash
# convh / convhw microbench (tools/convh_bench.py) with per-kernel times, then one SQ PMC pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/convh
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ch -o run --output-format csv -- python3 "$R/tools/convh_bench.py" \
  > "$OUT/bench.md" 2>&1 || { tail -30 "$OUT/bench.md"; exit 1; }
grep "|\|rel" "$OUT/bench.md"
f=$(find /tmp/ch -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kstats.csv"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d /tmp/chp -o run -- python3 "$R/tools/convh_bench.py" --reps 2 > "$OUT/pmc.log" 2>&1 || exit $?
f=$(find /tmp/chp -name "*counter_collection.csv" | head -1); cp "$f" "$OUT/pmc1.csv"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_VALU SQ_INSTS_SALU \
  --output-format csv -d /tmp/chp2 -o run -- python3 "$R/tools/convh_bench.py" --reps 2 > "$OUT/pmc2.log" 2>&1 || exit $?
f=$(find /tmp/chp2 -name "*counter_collection.csv" | head -1); cp "$f" "$OUT/pmc2.csv"
echo done
