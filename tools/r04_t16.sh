# does the k-shard factor chain share a hardware queue with the y build?  emulated 8 ranks at
# GPU_MAX_HW_QUEUES 4 (the box default) / 8 / 16, and the 1-GPU step at 4 / 8
set -o pipefail
for i in 1 2; do
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t16_emu_q${q}_$i.json 2> gpurun_out/r04_t16_emu_q${q}_$i.err || { echo FAIL $q; tail -5 gpurun_out/r04_t16_emu_q${q}_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04_t16_emu_q${q}_$i.json').read().strip().splitlines()[-1])
r=[x for x in d['ranks'] if x['rank']==d['worst_rank']][0]
print('queues $q run $i max', d['max_rank_ms'], 'worst', d['worst_rank'], {k: r['stages_ms'][k] for k in ('select','x4','y','factor','fft','trsm','herk')})"
done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t16_b_q${q}_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04_t16_b_q${q}_$i.json').read().strip().splitlines()[-1]); print('1gpu queues $q run $i', d['ms_per_step'])"
done
done
exit 0
