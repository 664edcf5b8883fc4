#!/bin/bash
# One build-measure iteration: the named GPU test files, optional microbench, then the ResNet-50
# b1024 bench under rocprofv3 (per-kernel summary + autotune decisions).
# Usage: scripts/gpu_iter.sh TAG "tests/test_a.py tests/test_b.py" [tool.py ...]
set -o pipefail
TAG=$1; TESTS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -40 "$OUT/tests.txt"; exit 1; }
  tail -2 "$OUT/tests.txt"
fi
for t in "$@"; do
  timeout -k 10 300 python "$t" > "$OUT/$(basename "$t" .py).md" 2>&1 || { cat "$OUT/$(basename "$t" .py).md"; exit 1; }
  cat "$OUT/$(basename "$t" .py).md"
done
PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh ${TAG}_resnet50 --steps 10 --warmup 5 || exit $?
head -22 "$R/gpurun_out/prof_${TAG}_resnet50/summary.md"
python3 -c "import json;d=json.load(open('$R/gpurun_out/prof_${TAG}_resnet50/bench.json'));print(d['value'],d['ms_per_step'],d['final_loss'],d['params_finite'],d['autotune'])"
