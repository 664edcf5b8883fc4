#!/bin/bash
# GEMM timing table (ours vs hipBLASLt) + rocprofv3 PMC passes over one of our GEMMs.
# Usage: scripts/gpu_gemm_pmc.sh TAG LAYOUTxMxNxK
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; SHAPE=${2:-NTx4096x4096x4096}
OUT=$R/gpurun_out/gemm_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/tools/gemm_probe.py" --shapes all > "$OUT/table.md" 2> "$OUT/table.err" || exit $?
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16" \
           "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/gpmc$i -o run -- python3 "$R/tools/gemm_probe.py" \
    --pmc "$SHAPE" > "$OUT/pmc$i.log" 2>&1 || exit $?
  f=$(find /tmp/gpmc$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/pass$i.csv"
done
exit 0
