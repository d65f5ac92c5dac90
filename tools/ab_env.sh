#!/bin/bash
# Interleaved A/B of one environment knob on the C3 bench (no CPU baseline, no isolated step):
#   bash tools/ab_env.sh ROUNDS VAR v1 v2 ...     prints ms/step and the stage split per value
set -o pipefail
R=$1; VAR=$2; shift 2
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for v in "$@"; do
    env "$VAR=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-isolated $BENCH_ARGS \
      > gpurun_out/ab/$VAR.$v.$i.json 2> gpurun_out/ab/$VAR.$v.$i.err || { tail -20 gpurun_out/ab/$VAR.$v.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; r=d['roofline']; print(sys.argv[2], d['ms_per_step'], 'trsm/launch', round(r['avg_launch_ms'],3) if r['kernel'].startswith('zgemm_glds_kernel<0,0') else r, {k: s[k] for k in ('select','y','factor','fft','trsm','herk','small')})" gpurun_out/ab/$VAR.$v.$i.json "$VAR=$v"
  done
done
