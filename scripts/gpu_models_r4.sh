#!/bin/bash
# the other BASELINE models on the current tree (no profiler): BERT-base b256, WRN-101-2 fp8 b512
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/models_r4
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bert.json" > "$OUT/bert.log" 2>&1 || { tail -20 "$OUT/bert.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bert.json'));print('bert', d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'])"
timeout -k 10 600 python3 bench.py --model wide_resnet101_2 --steps 10 --warmup 3 --out "$OUT/wrn.json" > "$OUT/wrn.log" 2>&1 || { tail -20 "$OUT/wrn.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/wrn.json'));print('wrn', d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'], d.get('dtype'))"
