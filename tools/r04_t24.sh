# HERK split-K reduce with 16 loads in flight per thread: kernels + shard parity, then timing
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_shard_full.py > gpurun_out/r04_t24_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t24_tests.log; exit 1; }
tail -1 gpurun_out/r04_t24_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t24_emu_$i.json 2>/dev/null || { echo FAIL emu; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t24_b_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
  python3 -c "
import json
e=json.loads(open('gpurun_out/r04_t24_emu_$i.json').read().strip().splitlines()[-1])
b=json.loads(open('gpurun_out/r04_t24_b_$i.json').read().strip().splitlines()[-1])
print('run $i: emu max', e['max_rank_ms'], [x['ms_per_step'] for x in e['ranks']], '| 1gpu', b['ms_per_step'], 'herk', b['stages_ms_per_step']['herk'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_t24_prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/r04_t24_prof.json 2> gpurun_out/r04_t24_prof.err
grep -i "herk_reduce" gpurun_out/r04_t24_prof/run_kernel_stats.csv | cut -c1-200
exit 0
