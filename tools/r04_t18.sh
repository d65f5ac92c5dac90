# real-A GEMM for the self-conjugate q's U = L^-1 Yhat: parity at full size, then A/B
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_shard_full.py > gpurun_out/r04_t18_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t18_tests.log; exit 1; }
tail -2 gpurun_out/r04_t18_tests.log
grep -i "dJ\|rel" gpurun_out/r04_t18_tests.log | head -20
for i in 1 2; do
for rt in 1 0; do
  FISDF_REAL_TRSM=$rt timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/r04_t18_b_r${rt}_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04_t18_b_r${rt}_$i.json').read().strip().splitlines()[-1]); print('real_trsm $rt run $i', d['ms_per_step'], 'trsm', d['stages_ms_per_step']['trsm'], 'iso', d['roofline']['isolated'])"
done
done
exit 0
