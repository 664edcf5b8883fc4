#!/bin/bash
# Round-6 call E: persistent vs one-workgroup-per-tile 8-phase GEMMs in the real step (feature
# gemm_persistent) on BERT-base and ResNet-50.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
ABTAG=persist_bert bash scripts/gpu_ab_env.sh gemm_persistent "1 0 1 0" --model bert_base || exit 1
ABTAG=persist_r50 bash scripts/gpu_ab_env.sh gemm_persistent "1 0" || exit 1
