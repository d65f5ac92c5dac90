# x4 through the register k-mesh DFT pair: parity (x4 vs oracle both ways, full-size configs,
# the 8-rank shard test, the C-ABI), then A/B against the dense Phi GEMMs
set -o pipefail
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_gpu_isdf.py tests/test_gpu_capi.py tests/test_gpu_configs.py tests/test_gpu_shard_full.py > gpurun_out/r04_t22_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t22_tests.log; exit 1; }
tail -1 gpurun_out/r04_t22_tests.log
grep "x4 time_reversal\|c3: oracle\|c2: oracle\|c4: oracle\|c5: oracle\|rank regime: GPU\|displaced" gpurun_out/r04_t22_tests.log | head -20
for i in 1 2; do
for xd in 1 0; do
  FISDF_X4_DFT=$xd timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t22_emu_x${xd}_$i.json 2>/dev/null || { echo FAIL emu; exit 1; }
  FISDF_X4_DFT=$xd timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t22_b_x${xd}_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
  python3 -c "
import json
e=json.loads(open('gpurun_out/r04_t22_emu_x${xd}_$i.json').read().strip().splitlines()[-1])
b=json.loads(open('gpurun_out/r04_t22_b_x${xd}_$i.json').read().strip().splitlines()[-1])
print('x4_dft $xd run $i: emu max', e['max_rank_ms'], 'x4', e['ranks'][0]['stages_ms']['x4'], '| 1gpu', b['ms_per_step'], 'x4', b['stages_ms_per_step']['x4'])"
done
done
exit 0
