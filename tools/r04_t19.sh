set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "dgemm_real_a or modes_wide" > gpurun_out/r04_t19_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t19_tests.log; exit 1; }
tail -1 gpurun_out/r04_t19_tests.log
timeout -k 10 200 python -u tools/trsm_bench.py 2>&1 | grep -v amdgpu.ids
