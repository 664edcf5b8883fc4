#!/bin/bash
# Round-6 roofline table: a plain run pins the autotune decisions, then three
# rocprofv3 --pmc passes over the same ResNet-50 b1024 bench (one counter group per run, each with
# the kernel trace), summarised per kernel by tools/roofline.py. Usage: scripts/gpu_r6_roofline.sh TAG [bench args]
set -o pipefail
TAG=${1:-roof}; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
PSD_AUTOTUNE_SAVE=$OUT/decisions.json timeout -k 10 300 python3 bench.py --steps 3 --warmup 3 "$@" \
  --out "$OUT/bench_plain.json" > "$OUT/plain.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" \
           "FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "WRITE_SIZE SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i + 1))
  PSD_AUTOTUNE_FILE=$OUT/decisions.json timeout -s KILL 420 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
    -d /tmp/roof$i -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 "$@" > "$OUT/pass$i.log" 2>&1 || exit $?
  f=$(find /tmp/roof$i -name "*counter_collection.csv" | head -1)
  tr=$(find /tmp/roof$i -name "*kernel_trace.csv" | head -1)
  [ -n "$f" ] && gzip -c "$f" > "$OUT/pass$i.csv.gz"
  [ $i -eq 1 ] && [ -n "$tr" ] && gzip -c "$tr" > "$OUT/trace1.csv.gz"
  echo "pass $i done"
done
python3 "$R/tools/roofline.py" --trace "$OUT/trace1.csv.gz" "$OUT"/pass*.csv.gz --steps 2 --title "$TAG" > "$OUT/roofline.md"
cat "$OUT/roofline.md"
