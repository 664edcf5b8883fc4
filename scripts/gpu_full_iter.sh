#!/bin/bash
# The full GPU test suite, then the ResNet-50 b1024 bench under rocprofv3 (per-kernel summary +
# autotune decisions). Usage: scripts/gpu_full_iter.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -60 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh ${TAG}_resnet50 --steps 10 --warmup 5 "$@" || exit $?
head -30 "$R/gpurun_out/prof_${TAG}_resnet50/summary.md"
python3 -c "import json;d=json.load(open('$R/gpurun_out/prof_${TAG}_resnet50/bench.json'));print(d['value'],d['ms_per_step'],d['final_loss'],d['params_finite'],d['autotune'],d.get('autotune_source'))"
