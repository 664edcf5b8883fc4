#!/bin/bash
# same-box A/B of one environment switch on the BERT bench: scripts/gpu_ab_bert.sh VAR "v0 v1 v0 v1"
set -o pipefail
VAR=$1; VALS=$2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/abb_$VAR
mkdir -p "$OUT"
cd "$R"
i=0
for v in $VALS; do
  i=$((i+1))
  env "$VAR=$v" timeout -k 10 300 python3 bench.py --model bert_base --steps 30 --warmup 5 --out "$OUT/b$i.json" > "$OUT/b$i.log" 2>&1 || { tail -20 "$OUT/b$i.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b$i.json'));print('$VAR=$v', d['value'], d['ms_per_step'], d['final_loss'])"
done
