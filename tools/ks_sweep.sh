#!/bin/bash
# Step time vs HERK split-K (FISDF_HERK_KS) and fit lanes (FISDF_FIT_LANES) on the C3 bench.
# Usage: bash tools/ks_sweep.sh "ks:lanes" ...   (default: 41:2 24:2 60:2 41:3 24:3 41:2)
set -o pipefail
mkdir -p gpurun_out/ks
cfgs=("$@")
[ ${#cfgs[@]} -eq 0 ] && cfgs=(41:2 24:2 60:2 41:3 24:3 41:2)
i=0
for cfg in "${cfgs[@]}"; do
  ks=${cfg%%:*}; lanes=${cfg##*:}; i=$((i+1))
  out=gpurun_out/ks/b_${i}_${ks}_${lanes}.json
  FISDF_HERK_KS=$ks FISDF_FIT_LANES=$lanes timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 > $out 2> gpurun_out/ks/e_${i}.log || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('ks=$ks lanes=$lanes', d['ms_per_step'])" $out
done
