#!/bin/bash
# Round-6 call G: async PS at world 1 on plain device memory vs uncached IPC memory (feature
# async_cached_local) on BERT-base and ResNet-50, after the async GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r6g
timeout -k 10 400 python -u -m pytest tests/test_async_ps.py tests/test_stream_census.py -m gpu -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/r6g/async_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6g/async_tests.txt; [ $rc -eq 0 ] || exit $rc
ABTAG=cached_bert bash scripts/gpu_ab_env.sh async_cached_local "1 0 1 0" --model bert_base || exit 1
ABTAG=cached_r50 bash scripts/gpu_ab_env.sh async_cached_local "1 0 1 0" || exit 1
