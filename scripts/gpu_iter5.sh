#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash scripts/gpu_iter4.sh || exit $?
bash scripts/gpu_models_r4.sh || exit $?
