# WHAT-IF: how much of each emulated rank the replicated selection holds (points handed over)
set -o pipefail
for i in 1 2; do
for w in 0 1; do
  FISDF_WHATIF_GIVEN_X=$w timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t30_w${w}_$i.json 2>/dev/null || { echo FAIL; exit 1; }
  python3 -c "
import json; e=json.loads(open('gpurun_out/r04_t30_w${w}_$i.json').read().strip().splitlines()[-1]); print('given_x $w run $i max', e['max_rank_ms'], [x['ms_per_step'] for x in e['ranks']])"
done
done
exit 0
