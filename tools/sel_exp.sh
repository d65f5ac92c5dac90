#!/bin/bash
# Timing experiments on the cooperative selection kernel (C3, select_bench + phase probe):
#   bash tools/sel_exp.sh TAG "ENV=v ..." ["ENV=v ..." ...]     (each argument one variant;
#   FISDF_LIB_VARIANT=name loads fisdf/libfisdf_name.so from tools/build_variant.sh)
set -o pipefail
OUT=gpurun_out/${1:-selexp}; shift
mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i + 1))
  env $v FISDF_SEL_MODE=coop timeout -k 10 120 python -u tools/select_bench.py --cfg c3 > $OUT/sb_$i.log 2>&1 || { echo "FAIL [$v]"; tail -5 $OUT/sb_$i.log; exit 1; }
  env $v FISDF_SEL_PROF=1 FISDF_SEL_MODE=coop timeout -k 10 120 python -u tools/select_bench.py --cfg c3 --reps 1 > $OUT/sbp_$i.log 2>&1 || exit 1
  echo "[$v] $(tail -1 $OUT/sb_$i.log | cut -c30-90) | $(grep 'select coop' $OUT/sbp_$i.log | tail -1)"
done
