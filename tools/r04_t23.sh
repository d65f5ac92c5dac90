# one-call W_s row blocks (fisdf_build_ws_blocks): sharded parity, then the emulated 8-rank step
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_shard_full.py tests/test_gpu_rccl.py tests/test_gpu_dist.py > gpurun_out/r04_t23_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t23_tests.log; exit 1; }
tail -1 gpurun_out/r04_t23_tests.log
grep "sum of W_s" gpurun_out/r04_t23_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t23_emu_$i.json 2>/dev/null || { echo FAIL emu; exit 1; }
  python3 -c "
import json
e=json.loads(open('gpurun_out/r04_t23_emu_$i.json').read().strip().splitlines()[-1])
print('run $i: emu max', e['max_rank_ms'], [x['ms_per_step'] for x in e['ranks']], 'ws', e['ranks'][4]['stages_ms']['ws'])"
done
exit 0
