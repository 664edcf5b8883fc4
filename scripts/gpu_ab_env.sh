#!/bin/bash
# same-box A/B of one kernel-path feature (utils/config.py FEATURES) on the ResNet-50 bench:
#   scripts/gpu_ab_env.sh FEATURE "1 0 1 0" [bench args]
set -o pipefail
F=$1; VALS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/ab_${ABTAG:-$F}
mkdir -p "$OUT"
cd "$R"
i=0
for v in $VALS; do
  i=$((i+1))
  PSD_FEATURES="$F=$v" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 "$@" --out "$OUT/b$i.json" > "$OUT/b$i.log" 2>&1 || { tail -20 "$OUT/b$i.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b$i.json'));print('$F=$v', d['value'], d['ms_per_step'], d['final_loss'])"
done
