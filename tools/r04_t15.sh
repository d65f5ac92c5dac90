# k-shard y build on a CU-masked stream (FISDF_Y_FREE_CUS CUs left to the factor chain): emulated 8 ranks
set -o pipefail
for i in 1 2; do
for n in 0 32 64 16 128; do
  FISDF_Y_FREE_CUS=$n timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t15_emu_f${n}_$i.json 2> gpurun_out/r04_t15_emu_f${n}_$i.err || { echo FAIL $n; tail -5 gpurun_out/r04_t15_emu_f${n}_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04_t15_emu_f${n}_$i.json').read().strip().splitlines()[-1])
r=[x for x in d['ranks'] if x['rank']==d['worst_rank']][0]
print('free $n run $i max', d['max_rank_ms'], 'worst', d['worst_rank'], {k: r['stages_ms'][k] for k in ('y','factor','trsm','herk')})"
done
done
exit 0
