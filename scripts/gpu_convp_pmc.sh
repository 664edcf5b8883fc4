#!/bin/bash
# PMC passes over the persistent 1x1 kernel's statistics-only / apply passes (layer1 tail shape)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/convp_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for ps in stats apply; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
    --output-format csv -d /tmp/cp1_$ps -o run -- python3 "$R/tools/convp_probe.py" --pass $ps > "$OUT/p1_$ps.log" 2>&1 || exit $?
  f=$(find /tmp/cp1_$ps -name "*counter_collection.csv" | head -1); cp "$f" "$OUT/p1_$ps.csv"
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT \
    --output-format csv -d /tmp/cp2_$ps -o run -- python3 "$R/tools/convp_probe.py" --pass $ps > "$OUT/p2_$ps.log" 2>&1 || exit $?
  f=$(find /tmp/cp2_$ps -name "*counter_collection.csv" | head -1); cp "$f" "$OUT/p2_$ps.csv"
done
cd "$R" && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/cpt -o run --output-format csv -- python3 tools/convp_probe.py --pass stats > "$OUT/trace.log" 2>&1
f=$(find /tmp/cpt -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kstats.csv"; cut -c1-150 "$OUT/kstats.csv" | head -5
echo done
