#!/bin/bash
# async S=1 with 1 vs 2 push streams (hardware-queue sharing), and sync S=0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/adiag3
mkdir -p "$OUT"
cd "$R"
run() {
  tag=$1; shift
  env "$@" PSD_STEP_LOG=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/$tag.json" > "$OUT/$tag.log" 2>&1 || { tail -20 "$OUT/$tag.log"; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['staleness_hist'])"
  grep "step host ms" "$OUT/$tag.log" | cut -c1-120
}
run async_1stream PSD_ASYNC_PUSH_STREAMS=1 || exit 1
run async_2stream PSD_ASYNC_PUSH_STREAMS=2 || exit 1
run async_1stream_tail PSD_ASYNC_PUSH_STREAMS=1 PSD_TAIL_RECOMPUTE=1 || exit 1
exit 0
