#!/bin/bash
# Interleaved A/B of library variants x hardware-queue counts on the C3 bench:
#   bash tools/ab_hwq.sh ROUNDS "HWQ:variant" ...   ("default" = libfisdf.so)
# HIP spreads a process's streams over GPU_MAX_HW_QUEUES hardware queues (4 by default); streams
# sharing a queue run their kernels in submission order.
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for c in "$@"; do
    q=${c%%:*}; v=${c#*:}; vv=$v; [ "$v" = "default" ] && vv=""
    GPU_MAX_HW_QUEUES=$q FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-isolated $BENCH_ARGS \
      > gpurun_out/ab/q$q.$v.$i.json 2> gpurun_out/ab/q$q.$v.$i.err || { tail -20 gpurun_out/ab/q$q.$v.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; print(sys.argv[2], d['ms_per_step'], {k: s[k] for k in ('select','y','factor','fft','trsm','herk','small')})" gpurun_out/ab/q$q.$v.$i.json "hwq=$q $v"
  done
done
