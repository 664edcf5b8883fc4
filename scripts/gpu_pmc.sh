#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, --kernel-trace-free) over tools/kernel_pmc.py;
# leaves per-kernel counter tables in gpurun_out/pmc/. Usage: scripts/gpu_pmc.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc$i -o run -- python3 "$R/tools/kernel_pmc.py" \
    > "$OUT/run$i.log" 2>&1 || exit $?
  f=$(find /tmp/pmc$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/pass$i.csv"
done
exit 0
