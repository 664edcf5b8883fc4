set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stem2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/st2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stem_bench.py > $GRAFT_REPO_ROOT/gpurun_out/stem2/bench.md 2>&1 || { cat $GRAFT_REPO_ROOT/gpurun_out/stem2/bench.md; exit 1; }
cat $GRAFT_REPO_ROOT/gpurun_out/stem2/bench.md
f=$(find /tmp/st2 -name "*kernel_stats.csv" | head -1); cp "$f" $GRAFT_REPO_ROOT/gpurun_out/stem2/kstats.csv
cut -d, -f1-8 $GRAFT_REPO_ROOT/gpurun_out/stem2/kstats.csv | head -20
