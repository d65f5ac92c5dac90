set -o pipefail
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_shard_full.py "tests/test_gpu_configs.py::test_end_to_end_own_selection" > gpurun_out/r04_t2.log 2>&1 || { echo FAIL tests; exit 1; }
timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_emulate8.json 2> gpurun_out/r04_emulate8.err || { echo FAIL emu; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench_base.json 2> gpurun_out/r04_bench_base.err
