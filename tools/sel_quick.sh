#!/bin/bash
# C3 select_bench of the cooperative kernel per FISDF_SEL_REG value, pivots compared, phase probe.
#   bash tools/sel_quick.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-selq}
mkdir -p $OUT
for reg in 1 0 1 0; do
  FISDF_SEL_MODE=coop FISDF_SEL_REG=$reg timeout -k 10 120 python -u tools/select_bench.py --cfg c3 --save $OUT/piv_$reg.npz > $OUT/sb_$reg.log 2>&1 || { echo "BENCH FAILED $reg"; tail -5 $OUT/sb_$reg.log; exit 1; }
  echo "reg=$reg $(tail -1 $OUT/sb_$reg.log)"
done
for reg in 1 0; do
  FISDF_SEL_PROF=1 FISDF_SEL_MODE=coop FISDF_SEL_REG=$reg timeout -k 10 120 python -u tools/select_bench.py --cfg c3 --reps 1 > $OUT/sbp_$reg.log 2>&1 || { echo "PROBE FAILED"; exit 1; }
  echo "reg=$reg $(grep 'select coop' $OUT/sbp_$reg.log | tail -1)"
done
python3 -c "
import numpy as np
a=np.load('$OUT/piv_1.npz')['perm']; b=np.load('$OUT/piv_0.npz')['perm']
print('c3 reg vs lds pivots identical:', a.shape == b.shape and bool((a == b).all()), len(a))"
