#!/bin/bash
# PMC passes over our GEMM for several shapes (tools/gemm_probe.py --pmc, 5 launches each), summarised
# by tools/pmc_summary.py. Usage: scripts/gpu_r6_gpmc.sh TAG SHAPE [SHAPE ...]   (SHAPE = LAYOUTxMxNxK)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/gpmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for SHAPE in "$@"; do
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16" \
             "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d /tmp/gp_${SHAPE}_$i -o run -- \
      python3 "$R/tools/gemm_probe.py" --pmc "$SHAPE" > "$OUT/${SHAPE}_$i.log" 2>&1 || exit $?
    f=$(find /tmp/gp_${SHAPE}_$i -name "*counter_collection.csv" | head -1)
    [ -n "$f" ] && cp "$f" "$OUT/${SHAPE}_pass$i.csv"
  done
  python3 "$R/tools/pmc_summary.py" "$OUT/${SHAPE}"_pass*.csv --kernel gemm8p > "$OUT/${SHAPE}.md" 2>&1
  echo "== $SHAPE"; tail -8 "$OUT/${SHAPE}.md"
done
exit 0
