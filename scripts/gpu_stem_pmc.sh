#!/bin/bash
# stem passes (tools/stem_bench.py) under two SQ / TA PMC passes: where the stem conv and its weight
# gradient spend their cycles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/stempmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/tools/stem_bench.py" --reps 3 > "$OUT/bench.md" 2>&1 || { tail -20 "$OUT/bench.md"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d /tmp/sp1 -o run -- python3 "$R/tools/stem_bench.py" --reps 1 > "$OUT/pmc1.log" 2>&1 || exit $?
f=$(find /tmp/sp1 -name "*counter_collection.csv" | head -1); cp "$f" "$OUT/pmc1.csv"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_VALU SQ_INSTS_SALU \
  --output-format csv -d /tmp/sp2 -o run -- python3 "$R/tools/stem_bench.py" --reps 1 > "$OUT/pmc2.log" 2>&1 || exit $?
f=$(find /tmp/sp2 -name "*counter_collection.csv" | head -1); cp "$f" "$OUT/pmc2.csv"
cat "$OUT/bench.md" | grep "|"
echo done
