#!/bin/bash
# final round-4 numbers on the default tree: ResNet-50 (headline), BERT-base, WRN-101-2 fp8
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/final_bench
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/resnet.json" > "$OUT/resnet.log" 2>&1 || { tail -20 "$OUT/resnet.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/resnet.json'));print('resnet', d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'])"
bash scripts/gpu_models_r4.sh
