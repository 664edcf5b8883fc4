#!/bin/bash
# BERT-base b256 profile with autotune timings (linear fwd / dgrad / wgrad: mfma vs hipBLASLt)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh bert_r4 --model bert_base --steps 10 --warmup 5 || exit $?
head -40 "$R/gpurun_out/prof_bert_r4/summary.md"
grep "autotune\]" "$R/gpurun_out/prof_bert_r4/run.log" | grep linear | cut -c1-220
python3 -c "import json;d=json.load(open('$R/gpurun_out/prof_bert_r4/bench.json'));print(d['value'],d['ms_per_step'],d['final_loss'],d['params_finite'])"
