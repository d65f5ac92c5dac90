#!/bin/bash
# Selection kernels on one box: the GPU selection tests (batch kernel = default), then C3 (and C4)
# timing of each mode with the per-batch / per-step phase probe, and the pivots compared.
#   bash tools/sel_ab.sh TAG
set -o pipefail
TAG=${1:-sel}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_selection.py "tests/test_gpu_isdf.py::test_selection_paths_agree" > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|^E " $OUT/tests.log | tail -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
grep -E "identical prefix|tie at" $OUT/tests.log | cut -c1-160
for cfg in c3 c4; do
  for mode in coop batch; do
    FISDF_SEL_MODE=$mode timeout -k 10 120 python -u tools/select_bench.py --cfg $cfg --save $OUT/piv_${cfg}_$mode.npz > $OUT/sb_${cfg}_$mode.log 2>&1 || { echo "BENCH FAILED $cfg $mode"; tail -5 $OUT/sb_${cfg}_$mode.log; exit 1; }
    tail -1 $OUT/sb_${cfg}_$mode.log
    FISDF_SEL_PROF=1 FISDF_SEL_MODE=$mode timeout -k 10 120 python -u tools/select_bench.py --cfg $cfg --reps 1 > $OUT/sbp_${cfg}_$mode.log 2>&1 || { echo "PROBE FAILED"; exit 1; }
    grep "select " $OUT/sbp_${cfg}_$mode.log | tail -1
  done
  python3 -c "
import numpy as np
a=np.load('$OUT/piv_${cfg}_coop.npz')['perm']; b=np.load('$OUT/piv_${cfg}_batch.npz')['perm']
n=min(len(a),len(b)); same=(a[:n]==b[:n]); print('$cfg coop vs batch: len', len(a), len(b), 'identical prefix', int(np.argmin(same)) if not same.all() else n)"
done
