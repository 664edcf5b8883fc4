#!/bin/bash
# same-box A/B of the async transport at N = 1: scatter / gather kernels vs hipMemcpyAsync
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/xfer_ab
mkdir -p "$OUT"
cd "$R"
for m in bert_base resnet50; do
  for x in kernel copy kernel copy; do
    timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 --async-xfer $x --out "$OUT/${m}_$x.json" > "$OUT/${m}_$x.log" 2>&1 || { tail -20 "$OUT/${m}_$x.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${m}_$x.json'));print('$m $x', d['value'], d['ms_per_step'], d['config']['async_xfer'])"
  done
done
