#!/bin/bash
# WRN-101-2 fp8: MX vs per-tensor scaling, same box, AB (async plane). Usage: scripts/gpu_ab_wrn.sh TAG
set -o pipefail
TAG=${1:-wrn}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p "$OUT"
cd "$R"
for side in A B; do
  if [ $side = A ]; then E=PSD_FEATURES=fp8_mx=0; else E=PSD_FEATURES=fp8_mx=1; fi
  env $E timeout -k 10 400 python3 bench.py --model wide_resnet101_2 --steps 10 --warmup 3 --out "$OUT/$side.json" > "$OUT/$side.log" 2>&1 || { tail -20 "$OUT/$side.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$side.json'));print('$side [$E]:', d['value'], 'img/s', d['ms_per_step'], 'ms loss', d['final_loss'], d['params_finite'])"
done
