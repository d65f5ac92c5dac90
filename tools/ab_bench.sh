#!/bin/bash
# Interleaved A/B of library builds on the C3 bench (no CPU baseline, no isolated step):
#   bash tools/ab_bench.sh ROUNDS v1 v2 ...   ("default" = libfisdf.so, else libfisdf_<v>.so)
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for v in "$@"; do
    vv=$v; [ "$v" = "default" ] && vv=""
    FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-isolated $BENCH_ARGS \
      > gpurun_out/ab/$v.$i.json 2> gpurun_out/ab/$v.$i.err || { tail -20 gpurun_out/ab/$v.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; print(sys.argv[2], d['ms_per_step'], {k: s[k] for k in ('select','y','factor','trsm','herk','small')})" gpurun_out/ab/$v.$i.json $v
  done
done
