#!/bin/bash
# Round-6 round-end check on one box: the whole GPU suite, smoke(), the three BASELINE model benches
# (ResNet-50 twice) and the ResNet-50 / BERT-base kernel tables. Usage: scripts/gpu_r6_final.sh TAG
set -o pipefail
TAG=${1:-r6f}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -4 "$OUT/gpu_tests.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit $?
tail -1 "$OUT/smoke.txt"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --out "$OUT/bench_resnet50_$i.json" > "$OUT/bench_resnet50_$i.log" 2>&1 || exit $?
done
PSD_AUTOTUNE_LOG=1 timeout -k 10 300 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bench_bert.json" > "$OUT/bench_bert.log" 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --model wide_resnet101_2 --steps 20 --warmup 5 --out "$OUT/bench_wrn.json" > "$OUT/bench_wrn.log" 2>&1 || exit $?
python3 -c "
import json
for f in ('bench_resnet50_1', 'bench_resnet50_2', 'bench_bert', 'bench_wrn'):
    d = json.load(open('$OUT/' + f + '.json')); print(f, d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'])"
PSD_AUTOTUNE_LOG=1 bash scripts/gpu_profile_bench.sh ${TAG}_r50 --steps 10 --warmup 5 || exit $?
bash scripts/gpu_profile_bench.sh ${TAG}_bert --model bert_base --steps 10 --warmup 5 || exit $?
