#!/bin/bash
# Tune the library GEMMs of the bench models with PyTorch TunableOp on the GPU box and install the
# merged results as tuning/tunableop/gfx950.csv (copied to gpurun_out/ to be committed).
# Usage (on the box): bash scripts/tune_gemms.sh
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/tunableop
mkdir -p "$OUT" "$R/tuning/tunableop"
cd "$R"
timeout -k 10 400 python bench.py --model bert_base --steps 3 --warmup 3 --tunableop tune \
  --tunableop-out "$OUT/bert.csv" > "$OUT/bert.log" 2>&1
timeout -k 10 500 python bench.py --model resnet50 --steps 3 --warmup 3 --tunableop tune \
  --tunableop-out "$OUT/resnet50.csv" > "$OUT/resnet50.log" 2>&1
python -c "
from parameter_server_distributed_amd.utils import tunableop as t
n = t.merge(['$OUT/bert.csv', '$OUT/resnet50.csv'], '$R/tuning/tunableop/gfx950.csv')
print('tuned GEMMs:', n)"
cp "$R/tuning/tunableop/gfx950.csv" "$OUT/gfx950.csv"
