#!/bin/bash
# rocprofv3 PMC passes over tools/convn_pmc.py (layer1 narrow convolutions, every variant), one
# counter group per run; per-pass CSVs in gpurun_out/convn_pmc/. Usage: scripts/gpu_convn_pmc.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/convn_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum FETCH_SIZE" "WRITE_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "TA_TA_BUSY_sum TA_BUFFER_LOAD_WAVEFRONTS_sum TD_TD_BUSY_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/cpmc$i -o run -- python3 "$R/tools/convn_pmc.py" \
    > "$OUT/run$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i failed rc=$rc: $grp"; tail -5 "$OUT/run$i.log"
    case $rc in 124|134|137|139) exit $rc ;; esac  # a kill, abort or fault ends the script
    continue
  fi
  f=$(find /tmp/cpmc$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/pass$i.csv"
  echo "pass $i ok"
done
exit 0
