#!/bin/bash
# config 2 (sync SGD, staleness 0) next to the async default on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/sync_r4
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 bench.py --staleness 0 --steps 20 --warmup 5 --out "$OUT/sync.json" > "$OUT/sync.log" 2>&1 || { tail -20 "$OUT/sync.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/sync.json'));print('sync', d['value'], d['ms_per_step'], d['final_loss'], d['staleness_hist'])"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/async.json" > "$OUT/async.log" 2>&1 || { tail -20 "$OUT/async.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/async.json'));print('async', d['value'], d['ms_per_step'], d['final_loss'], d['staleness_hist'])"
