#!/bin/bash
# persistent prefetching attention kernels: tests + BERT bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/attn
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention.py tests/test_embedding.py tests/test_layernorm.py > "$OUT/tests.txt" 2>&1
rc=$?; tail -2 "$OUT/tests.txt"
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" "$OUT/tests.txt" | head -20; exit $rc; fi
timeout -k 10 400 python3 bench.py --model bert_base --steps 20 --warmup 5 --out "$OUT/bert.json" > "$OUT/bert.log" 2>&1 || { tail -20 "$OUT/bert.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bert.json'));print('bert', d['value'], d['ms_per_step'], d['final_loss'], d['params_finite'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_attn -o run --output-format csv -- python3 "$R/bench.py" --model bert_base --steps 5 --warmup 3 --out "$OUT/bert_prof.json" > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
T=$(find /tmp/prof_attn -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/prof_summary.py" "$T" --steps 3 --title attn --top 40 > "$OUT/summary.md"
grep -E "attn|wall" "$OUT/summary.md"
