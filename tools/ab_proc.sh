#!/bin/bash
# Cross-process A/B of the C3 bench (3 steps each, no CPU baseline): for settings that change
# how streams are created (priorities), which an in-process A/B would perturb.
# Usage: bash tools/ab_proc.sh TAG ROUNDS "name:VAR=val VAR=val" "name:..."
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    name=${cfg%%:*}; vars=${cfg#*:}
    env FISDF_NOOP=1 $vars timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-isolated > $OUT/${name}_$r.json 2> $OUT/${name}_$r.err || { echo "$name FAILED"; tail -5 $OUT/${name}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${name}_$r.json')); s=d['stages_ms_per_step']; print('$name', $r, d['ms_per_step'], 'x4', s['x4'], 'factor', s['factor'], 'y', s['y'])"
  done
done
