#!/bin/bash
# Same-box A/B of bench.py: alternates two environment settings (ABAB), prints img/s per run.
# Usage: scripts/gpu_ab.sh TAG "ENV_A" "ENV_B" [bench args...]   e.g. "PSD_FEATURES=bn_fold=0" "PSD_FEATURES=bn_fold=1"
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p "$OUT"
cd "$R"
for i in 1 2; do
  for side in A B; do
    if [ $side = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 "$@" --out "$OUT/${side}$i.json" > "$OUT/${side}$i.log" 2>&1 || { tail -20 "$OUT/${side}$i.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${side}$i.json'));print('$side [$E] run $i:', d['value'], 'img/s', d['ms_per_step'], 'ms', 'loss', d['final_loss'])"
  done
done
