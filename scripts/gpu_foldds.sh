#!/bin/bash
# downsample-BN fold (layer-1 dual tail): model-level tests, same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/foldds
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn.py tests/test_bnfold.py tests/test_tail.py > "$OUT/tests.txt" 2>&1
rc=$?; tail -2 "$OUT/tests.txt"
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" "$OUT/tests.txt" | head -20; exit $rc; fi
bash scripts/gpu_ab_env.sh PSD_BN_FOLD_DS "1 0 1 0"
