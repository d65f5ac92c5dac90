# selection kernel at 512 threads (16 threads per owned row): phase timing, the full GPU suite
# (pivots vs dpstrf, the displaced cells, the shard tests), then the emulated and 1-GPU steps
set -o pipefail
FISDF_LIB_VARIANT=sel512 FISDF_SEL_PROF=1 timeout -k 10 120 python -u tools/select_bench.py --reps 3 2>&1 | grep "select" || { echo PROBE FAILED; exit 1; }
FISDF_LIB_VARIANT=sel512 timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r04_t33_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04_t33_tests.log; exit 1; }
tail -1 gpurun_out/r04_t33_tests.log
grep "pivots identical\|identical prefix" gpurun_out/r04_t33_tests.log | cut -c1-150 | head -10
for i in 1 2; do
for v in sel512 default; do
  vv=$v; [ "$v" = "default" ] && vv=""
  FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t33_emu_${v}_$i.json 2>/dev/null || { echo FAIL emu; exit 1; }
  FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t33_b_${v}_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
  python3 -c "
import json
e=json.loads(open('gpurun_out/r04_t33_emu_${v}_$i.json').read().strip().splitlines()[-1])
b=json.loads(open('gpurun_out/r04_t33_b_${v}_$i.json').read().strip().splitlines()[-1])
print('$v run $i: emu max', e['max_rank_ms'], 'select', e['ranks'][4]['stages_ms']['select'], '| 1gpu', b['ms_per_step'], 'select', b['stages_ms_per_step']['select'])"
done
done
exit 0
