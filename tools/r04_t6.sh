set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread tests/test_gpu_shard_full.py tests/test_gpu_rccl.py tests/test_gpu_capi.py > gpurun_out/r04_t6_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t6_tests.log; exit 1; }
tail -3 gpurun_out/r04_t6_tests.log
for i in 1 2; do
for cfg in "FISDF_Y_PREFFT=0" "FISDF_Y_PREFFT=1" "FISDF_YPRE_BLOCKS=3" "FISDF_YPRE_BLOCKS=12"; do
  env $cfg timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t6_${cfg}_$i.json 2>/dev/null || echo "fail $cfg"
done
done
exit 0
