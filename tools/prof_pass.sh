#!/bin/bash
# One rocprofv3 PMC pass of the C3 bench (run each pass in its own gpurun call: the profiled
# process may crash in its exit handlers after the output is written).
# Usage: bash tools/prof_pass.sh TAG NAME COUNTER
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc $3 --output-format csv -d $OUT/$2 -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $OUT/$2.json 2> $OUT/$2.err
rc=$?
ls $OUT/$2/run_counter_collection.csv > /dev/null && echo "pass $2 rc=$rc output present"
exit $rc
