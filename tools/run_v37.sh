set -o pipefail
O=gpurun_out/r02_v37; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 -- python3 bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > $O/b.json 2> $O/b.err || true
find $O/prof -name "*kernel_stats.csv" | head -3
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp $f $O/c5_kernel_stats.csv && head -25 $O/c5_kernel_stats.csv | cut -d, -f1-5
