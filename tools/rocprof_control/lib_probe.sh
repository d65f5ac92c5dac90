#!/bin/bash
# The bench under rocprofv3 (kernel trace), with the selection's cooperative launch (default)
# and without it (FISDF_SEL_COOP=0: the blocked single-workgroup path): does the exit-time
# SIGSEGV follow the cooperative launch?   bash tools/rocprof_control/lib_probe.sh TAG
TAG=${1:-rocprof_lib}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for mode in coop noncoop; do
  if [ $mode = noncoop ]; then export FISDF_SEL_COOP=0; else unset FISDF_SEL_COOP; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$mode -o run -- python3 bench.py --no-cpu-baseline --no-isolated --steps 1 --warmup 0 > $OUT/$mode.out 2> $OUT/$mode.err
  rc=$?
  echo "$mode rc=$rc segv-lines $(grep -c SIGSEGV $OUT/$mode.err)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done
exit 0
