# spin vs blocking host waits on the build's critical path (selection read-back, factor verdict)
set -o pipefail
for i in 1 2; do
for sp in 1 0; do
  FISDF_HOST_SPIN=$sp timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t20_emu_s${sp}_$i.json 2> gpurun_out/r04_t20_emu_s${sp}_$i.err || { echo FAIL emu; tail -5 gpurun_out/r04_t20_emu_s${sp}_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04_t20_emu_s${sp}_$i.json').read().strip().splitlines()[-1])
print('spin $sp run $i emu max', d['max_rank_ms'], 'ranks', [x['ms_per_step'] for x in d['ranks']])"
  FISDF_HOST_SPIN=$sp timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t20_b_s${sp}_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04_t20_b_s${sp}_$i.json').read().strip().splitlines()[-1]); print('spin $sp run $i 1gpu', d['ms_per_step'])"
done
done
exit 0
