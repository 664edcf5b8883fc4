#!/bin/bash
# Round-6 call C: same-box A/Bs -- our kernels only (feature library_candidates 0) vs with the
# library candidates on ResNet-50 and BERT-base; the fp8 Wide-ResNet's identity blocks on the bf16
# recomputing tail (feature tail_fp8) -- and the fp8 tail test.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r6c
timeout -k 10 300 python -u -m pytest tests/test_fp8_training.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "tail or tracks" > gpurun_out/r6c/fp8_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r6c/fp8_tests.txt; [ $rc -eq 0 ] || exit $rc
ABTAG=libc_r50 bash scripts/gpu_ab_env.sh library_candidates "1 0 1 0" || exit 1
ABTAG=libc_bert bash scripts/gpu_ab_env.sh library_candidates "1 0 1 0" --model bert_base || exit 1
ABTAG=tail8_wrn bash scripts/gpu_ab_env.sh tail_fp8 "1 0" --model wide_resnet101_2 || exit 1
