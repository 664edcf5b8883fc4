#!/bin/bash
# Cross-rank consistency runs of the overlapped data plane with several ranks on one GPU (gloo).
# Usage: scripts/gpu_rank_check.sh TAG "<run args>" ["<run args>" ...]   (each quoted arg = one run)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/rankcheck_$TAG
mkdir -p "$OUT"
i=0
for args in "$@"; do
  i=$((i+1))
  NP=$(echo "$args" | sed -n 's/.*--np \([0-9]*\).*/\1/p'); NP=${NP:-2}
  RUNARGS=$(echo "$args" | sed 's/--np [0-9]*//')
  echo "run $i: np=$NP $RUNARGS" | tee -a "$OUT/index.txt"
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$NP" --master-addr 127.0.0.1 \
    --master-port $((29600 + i)) "$R/tools/rank_check.py" $RUNARGS --out "$OUT/run$i.jsonl" > "$OUT/run$i.log" 2>&1
  rc=$?
  echo "run $i rc=$rc" | tee -a "$OUT/index.txt"
  tail -1 "$OUT/run$i.jsonl" 2>/dev/null | tee -a "$OUT/index.txt"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
