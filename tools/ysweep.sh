#!/bin/bash
# y-build grid sub-block sweep (FISDF_YBLK_MB) on the C3 bench
for mb in 1024 256 128 64 32; do
  echo "YBLK_MB=$mb"
  FISDF_YBLK_MB=$mb timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 2 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms_per_step']['y'], d['stages_ms_per_step']['factor'])" || exit 1
done
