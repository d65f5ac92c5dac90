#!/bin/bash
# Round profile of the C3 bench on one MI355X: the default bench line (with CPU baseline), a
# rocprofv3 kernel trace of the warmup + timed steps only (--no-isolated: the untimed single-lane
# step is left out, so the CSV's per-step kernel time matches the bench's roofline), and
# FETCH_SIZE / WRITE_SIZE passes (separate runs) for the roofline kernels' HBM traffic.
#   bash tools/prof_round.sh TAG
# Until round 5 rocprofv3-profiled processes SIGSEGV'd in their exit handlers (ROCm 7.2's teardown
# of the state a cooperative launch leaves, profiles/r05/rocprof_exit/README.txt); since round 6
# the mirror launches the selection plainly and profiled runs exit 0.  Each pass is
# still judged by its output files; a timeout (124/137) stops the script.
set -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
ok() { local rc=$1 dir=$2 pat=$3; echo "pass $dir rc=$rc"; [ $rc -ne 124 ] && [ $rc -ne 137 ] && [ -n "$(find $dir -name "$pat" 2>/dev/null)" ]; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-isolated > $OUT/trace.json 2> $OUT/trace.err
ok $? $OUT/trace '*kernel_stats.csv' || { echo TRACE FAILED; tail -20 $OUT/trace.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --no-cpu-baseline --no-isolated --steps 1 --warmup 0 > $OUT/fetch.json 2> $OUT/fetch.err
ok $? $OUT/fetch '*counter_collection.csv' || { echo FETCH FAILED; tail -20 $OUT/fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --no-cpu-baseline --no-isolated --steps 1 --warmup 0 > $OUT/write.json 2> $OUT/write.err
ok $? $OUT/write '*counter_collection.csv' || { echo WRITE FAILED; tail -20 $OUT/write.err; exit 1; }
python3 tools/traffic.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json
