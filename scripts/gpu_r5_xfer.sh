#!/bin/bash
# round 5: async scatter/gather kernels -- GPU async tests (incl. world 8 on one GPU), fp8 PS tests,
# then the N=1 bench and a 2-rank rehearsal on the one GPU. Usage: scripts/gpu_r5_xfer.sh TAG
set -o pipefail
TAG=${1:-xfer}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_async_ps.py tests/test_fp8_ps.py tests/test_embedding.py > "$OUT/tests.txt" 2>&1 || { tail -60 "$OUT/tests.txt"; exit 1; }
tail -3 "$OUT/tests.txt"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/resnet.json" > "$OUT/resnet.log" 2>&1 || { tail -20 "$OUT/resnet.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/resnet.json'));print('resnet', d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'], d['config']['async_xfer'], d.get('async_plane_bw'))"
bash scripts/gpu_rehearsal.sh ${TAG}_rh || exit $?
for f in gpurun_out/${TAG}_rh/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'], d.get('final_loss'), d.get('params_finite'), d['config'].get('async_xfer'))"; done
