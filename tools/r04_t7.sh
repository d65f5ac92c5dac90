set -o pipefail
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_shard_full.py tests/test_gpu_rccl.py tests/test_gpu_dist.py > gpurun_out/r04_t7_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t7_tests.log; exit 1; }
tail -2 gpurun_out/r04_t7_tests.log
timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_emulate8_v2.json 2> gpurun_out/r04_emulate8_v2.err || { echo FAIL emu; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-isolated > gpurun_out/r04_t7_bench.json 2>/dev/null
