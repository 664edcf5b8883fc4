#!/bin/bash
# Round-6 call C2: the new GPU tests (fp8 tail, single-split GEMM), then BERT-base A/Bs
# (library_candidates, xfer_local) and the fp8 Wide-ResNet tail A/B (tail_fp8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r6c2
timeout -k 10 400 python -u -m pytest tests/test_fp8_training.py tests/test_gemm.py -m gpu -x -q --timeout 240 \
  --timeout-method thread -k "tail or tracks or single_split" > gpurun_out/r6c2/tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r6c2/tests.txt; [ $rc -eq 0 ] || exit $rc
ABTAG=libc_bert bash scripts/gpu_ab_env.sh library_candidates "1 0 1 0" --model bert_base || exit 1
ABTAG=xloc_bert bash scripts/gpu_ab_env.sh xfer_local "0 1" --model bert_base || exit 1
ABTAG=tail8_wrn bash scripts/gpu_ab_env.sh tail_fp8 "1 0" --model wide_resnet101_2 || exit 1
