#!/bin/bash
# One GPU call: parity tests, smoke, C3 bench (with CPU baseline), rocprofv3 kernel stats.
# Usage (from the repo root, on the GPU box): bash tools/gpu_check.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -rP > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
# the profiled process may crash in its exit handlers after rocprofv3 has written the
# stats (seen on this image); judge the pass by its output file
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/prof_bench.json 2> $OUT/prof.err
[ -n "$(find $OUT/prof -name '*kernel_stats.csv')" ] || { echo PROF FAILED; tail -30 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
head -25 $OUT/kernel_stats.csv | cut -c1-200
