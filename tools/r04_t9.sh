# speculative FFTs before the factor verdict: parity (sharded full-size, RCCL, dist, capi,
# displaced configs) then A/B timing, emulated 8 ranks and 1 GPU
set -o pipefail
timeout -k 10 800 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_shard_full.py tests/test_gpu_rccl.py tests/test_gpu_dist.py tests/test_gpu_capi.py tests/test_gpu_configs.py > gpurun_out/r04_t9_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t9_tests.log; exit 1; }
tail -2 gpurun_out/r04_t9_tests.log
for i in 1 2; do
for sp in 1 0; do
  FISDF_FIT_SPEC=$sp timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t9_emu_s${sp}_$i.json 2> gpurun_out/r04_t9_emu_s${sp}_$i.err || { echo FAIL emu; exit 1; }
  FISDF_FIT_SPEC=$sp timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t9_b_s${sp}_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
done
done
exit 0
