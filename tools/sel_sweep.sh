#!/bin/bash
# Sweep of the cooperative selection grid size (FISDF_SEL_WGS) on the C3 bench: select stage ms.
set -o pipefail
mkdir -p gpurun_out/sel
for g in 106 128 169 225 256; do
FISDF_SEL_WGS=$g timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/sel/b_$g.json 2> gpurun_out/sel/e_$g.log || exit 1
python -c "import json; d=json.load(open('gpurun_out/sel/b_$g.json')); print('wgs=$g', d['ms_per_step'], d['stages_ms_per_step']['select'])"
done
