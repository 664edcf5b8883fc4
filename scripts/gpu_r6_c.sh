#!/bin/bash
# Round-6 call C (ResNet-50): same-box A/Bs of our-kernels-only (feature library_candidates 0) and of
# own-shard pushes / pulls on the scatter kernel (feature xfer_local 1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
ABTAG=libc_r50 bash scripts/gpu_ab_env.sh library_candidates "1 0 1 0" || exit 1
ABTAG=xloc_r50 bash scripts/gpu_ab_env.sh xfer_local "0 1 0 1" || exit 1
