# the time-reversal-folded selection Gram: the full GPU suite, then the emulated 8-rank and the
# 1-GPU step
set -o pipefail
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r04_t31_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t31_tests.log; exit 1; }
tail -1 gpurun_out/r04_t31_tests.log
grep "dpstrf pivots identical\|tie\|own dpstrf" gpurun_out/r04_t31_tests.log | head -12
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t31_emu_$i.json 2>/dev/null || { echo FAIL emu; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t31_b_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
  python3 -c "
import json
e=json.loads(open('gpurun_out/r04_t31_emu_$i.json').read().strip().splitlines()[-1])
b=json.loads(open('gpurun_out/r04_t31_b_$i.json').read().strip().splitlines()[-1])
print('run $i: emu max', e['max_rank_ms'], 'select', e['ranks'][4]['stages_ms']['select'], '| 1gpu', b['ms_per_step'], 'select', b['stages_ms_per_step']['select'])"
done
exit 0
