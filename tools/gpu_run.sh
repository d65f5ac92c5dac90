#!/bin/bash
# One GPU call: a pytest selection, smoke, and the default bench line.
# Usage (repo root, on the GPU box): bash tools/gpu_run.sh TAG "PYTEST_ARGS" [bench-args|skip]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 1000 python -u -m pytest $2 -v --timeout 900 --timeout-method thread -rP \
    > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "PASSED|FAILED|ERROR|^E " $OUT/t.log | tail -40; tail -5 $OUT/t.log; exit 1; }
  tail -2 $OUT/t.log
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ "$3" != "skip" ]; then
  timeout -k 10 600 python -u bench.py $3 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
