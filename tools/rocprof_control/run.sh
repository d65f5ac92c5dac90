#!/bin/bash
# The rocprofv3 exit-crash controls, each under the profile command prof_round.sh uses
# (rocprofv3 --kernel-trace --stats), each with its own time limit:
#   A  ./control            C++ executable, one kernel, system HIP 7.2, no Python
#   B  python3 ctl.py        Python + ctypes libcontrol.so (system HIP 7.2), no torch, no libfisdf
#   C  python3 ctl.py --torch  Python + torch (its bundled HIP runtime), no libfisdf
#   D  ./control MAPS coop   (run.sh TAG coop) A plus one hipLaunchCooperativeKernel
# and the same three without the profiler.  Prints each exit status; the stderr tails and the
# maps go to gpurun_out/$TAG.
TAG=${1:-rocprof_control}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
D=tools/rocprof_control
run() {  # name, command...
  local name=$1; shift
  timeout -k 10 120 "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -c 'SIGSEGV' $OUT/$name.err) segv-lines"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && return 1
  return 0
}
if [ "$2" = "coop" ]; then  # D only: a cooperative launch under the profiler
  run D_plain $D/control $OUT/D_plain.maps coop || exit 1
  run D_prof rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/D -o run -- $D/control $OUT/D_prof.maps coop || exit 1
  exit 0
fi
run A_plain $D/control $OUT/A_plain.maps || exit 1
run B_plain python3 $D/ctl.py $OUT/B_plain.maps || exit 1
run C_plain python3 $D/ctl.py $OUT/C_plain.maps --torch || exit 1
run A_prof rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/A -o run -- $D/control $OUT/A_prof.maps || exit 1
run B_prof rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/B -o run -- python3 $D/ctl.py $OUT/B_prof.maps || exit 1
run C_prof rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/C -o run -- python3 $D/ctl.py $OUT/C_prof.maps --torch || exit 1
exit 0
