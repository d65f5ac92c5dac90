set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread tests/test_gpu_isdf.py -k "panels" tests/test_gpu_shard_full.py > gpurun_out/r04_t8_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t8_tests.log; exit 1; }
tail -2 gpurun_out/r04_t8_tests.log
for i in 1 2; do
for k in 1 4 8 2; do
  FISDF_FIT_PANELS=$k timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t8_p${k}_$i.json 2>/dev/null || echo "fail $k"
done
done
exit 0
