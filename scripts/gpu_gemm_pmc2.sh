#!/bin/bash
# PMC passes over one GEMM shape, ours vs hipBLASLt (tools/gemm_probe.py --pmc [--lib]).
# Usage: scripts/gpu_gemm_pmc2.sh TAG LAYOUTxMxNxK
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; SHAPE=$2
OUT=$R/gpurun_out/gpmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for who in ours lib; do
  extra=""; [ $who = lib ] && extra="--lib"
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE GRBM_COUNT" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/gp_${who}_$i -o run -- python3 "$R/tools/gemm_probe.py" \
      --pmc "$SHAPE" $extra > "$OUT/${who}_$i.log" 2>&1 || exit $?
    f=$(find /tmp/gp_${who}_$i -name "*counter_collection.csv" | head -1)
    [ -n "$f" ] && cp "$f" "$OUT/${who}_pass$i.csv"
    echo "done $who $i"
  done
done
exit 0
