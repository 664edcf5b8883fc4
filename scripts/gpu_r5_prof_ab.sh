#!/bin/bash
# rocprof kernel tables of the ResNet-50 bench with one feature on / off: scripts/gpu_r5_prof_ab.sh FEATURE
set -o pipefail
F=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh ${F}_on --steps 10 --warmup 5 || exit $?
PSD_FEATURES="$F=0" PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh ${F}_off --steps 10 --warmup 5 || exit $?
head -8 "$R/gpurun_out/prof_${F}_on/summary.md" | tail -2; head -8 "$R/gpurun_out/prof_${F}_off/summary.md" | tail -2
