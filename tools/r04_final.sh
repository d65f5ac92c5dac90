# round-end evidence of the final tree: the round profile (bench line with CPU baseline, kernel
# trace, FETCH/WRITE traffic), then the emulated 8-rank JSON (two runs)
set -o pipefail
bash tools/prof_round.sh r04_prof_v3 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_prof_v3/emulate8_$i.json 2>/dev/null || { echo FAIL emu; exit 1; }
  python3 -c "
import json; e=json.loads(open('gpurun_out/r04_prof_v3/emulate8_$i.json').read().strip().splitlines()[-1]); print('emu $i max', e['max_rank_ms'], [x['ms_per_step'] for x in e['ranks']])"
done
exit 0
