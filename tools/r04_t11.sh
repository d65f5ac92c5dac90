# pool-free temporaries + speculative FFTs: capi spec on/off, then the parity set
set -o pipefail
timeout -k 10 300 python -u tools/dbg/spec_capi.py toy222 > gpurun_out/r04_t11_dbg.log 2>&1 || { echo DBG FAILED; tail -20 gpurun_out/r04_t11_dbg.log; exit 1; }
cat gpurun_out/r04_t11_dbg.log
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_capi.py tests/test_gpu_shard_full.py tests/test_gpu_rccl.py tests/test_gpu_dist.py tests/test_gpu_configs.py tests/test_gpu_isdf.py > gpurun_out/r04_t11_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t11_tests.log; exit 1; }
tail -2 gpurun_out/r04_t11_tests.log
