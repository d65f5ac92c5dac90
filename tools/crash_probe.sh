#!/bin/bash
# VERDICT r05 #6, one GPU call.  (1) The group's exit-time core dump: fisdf_group with 3 ranks on
# GPU 0 (tests/capi_shard_worker.py group) with the cooperative-launch mutex dropped
# (FISDF_COOP_MUTEX=0), under tools/libcrashtrace.so (native backtrace + maps offsets of the
# faulting thread), then the same with the mutex.  (2) The stream -> hardware-queue mapping the HIP
# runtime logs (AMD_LOG_LEVEL=3) for a short bench with the cooperative launch and with the plain
# launch (FISDF_COOP_LAUNCH=0).  Usage: bash tools/crash_probe.sh TAG
set -o pipefail
TAG=${1:-crash_probe}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
W="import ctypes,runpy,sys; ctypes.CDLL('tools/libcrashtrace.so'); sys.argv=sys.argv[1:]; runpy.run_path(sys.argv[0], run_name='__main__')"
for m in 0 1; do
  D=$(mktemp -d)
  FISDF_COOP_MUTEX=$m FISDF_CRASH_OUT=$OUT/group_mutex$m.trace timeout -k 10 240 \
    python3 -u -c "$W" tests/capi_shard_worker.py toy331_fr 0 3 $D group > $OUT/group_mutex$m.log 2>&1
  echo "group mutex=$m rc=$?"
  [ -f $OUT/group_mutex$m.trace ] && grep -c crashtrace $OUT/group_mutex$m.trace
  rm -rf $D
done
for c in 1 0; do
  FISDF_Y_STREAM=0 FISDF_COOP_LAUNCH=$c AMD_LOG_LEVEL=3 timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --no-isolated > $OUT/bench_coop$c.json 2> $OUT/bench_coop$c.amdlog
  rc=$?
  echo "bench coop=$c rc=$rc"; cut -c1-300 $OUT/bench_coop$c.json
  grep -E "SWq|hardware queues|cooperative queue|HWq" $OUT/bench_coop$c.amdlog | cut -c1-400 > $OUT/queues_coop$c.txt
  wc -l $OUT/queues_coop$c.txt
  gzip -f $OUT/bench_coop$c.amdlog
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done
exit 0
