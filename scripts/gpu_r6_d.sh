#!/bin/bash
# Round-6 call D: the 8-phase GEMM's L2 warm-up (gemm_set_prefetch): GEMM tests, then the BERT-shape
# probe and the square reference with the warm-up on and off, then the ResNet-50 and BERT benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/r6d
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gemm.py -m gpu -x -q --timeout 180 --timeout-method thread \
  > "$OUT/gemm_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gemm_tests.txt"; [ $rc -eq 0 ] || exit $rc
for pf in 1 0 1; do
  PSD_GEMM_PF=$pf timeout -k 10 300 python3 tools/gemm_probe.py --shapes all > "$OUT/probe_pf$pf.md" 2>&1 || exit $?
done
paste -d'|' <(cut -d'|' -f1-6 "$OUT/probe_pf1.md") <(cut -d'|' -f6 "$OUT/probe_pf0.md") | head -40
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --out "$OUT/bench_r50.json" > "$OUT/bench_r50.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bench_bert.json" > "$OUT/bench_bert.log" 2>&1 || exit $?
python3 -c "
import json
for f in ('bench_r50', 'bench_bert'):
    d = json.load(open('$OUT/' + f + '.json')); print(f, d['value'], d['ms_per_step'])"
