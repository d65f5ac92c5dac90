# diagonal-block Cholesky with 1024 threads (2 x 2 per thread) vs 256 (4 x 4): kernel tests,
# the factor chain alone, the emulated 8-rank step and the 1-GPU step (FISDF_CHOL_TB 2 / 4)
set -o pipefail
FISDF_CHOL_TB=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "cholesky or tri_inverse" > gpurun_out/r04_t28_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t28_tests.log; exit 1; }
tail -1 gpurun_out/r04_t28_tests.log
for tb in 4 2; do FISDF_CHOL_TB=$tb timeout -k 10 200 python -u tools/factor_bench.py --batches 5 36 --reps 10 2>&1 | grep factor | sed "s/^/tb $tb /"; done
for i in 1 2; do
for tb in 2 4; do
  FISDF_CHOL_TB=$tb timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t28_emu_t${tb}_$i.json 2>/dev/null || { echo FAIL emu; exit 1; }
  python3 -c "
import json; e=json.loads(open('gpurun_out/r04_t28_emu_t${tb}_$i.json').read().strip().splitlines()[-1]); print('tb $tb run $i emu max', e['max_rank_ms'], [x['ms_per_step'] for x in e['ranks']], 'factor', e['ranks'][4]['stages_ms']['factor'])"
done
done
exit 0
