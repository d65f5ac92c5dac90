# round-end evidence of the final tree: smoke, the round profile, the emulated 8-rank JSON
set -o pipefail
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final3_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/r04_final3_smoke.log; exit 1; }
tail -1 gpurun_out/r04_final3_smoke.log
bash tools/prof_round.sh r04_prof_v5 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_prof_v5/emulate8_$i.json 2>/dev/null || { echo FAIL emu; exit 1; }
  python3 -c "
import json; e=json.loads(open('gpurun_out/r04_prof_v5/emulate8_$i.json').read().strip().splitlines()[-1]); print('emu $i max', e['max_rank_ms'], [x['ms_per_step'] for x in e['ranks']])"
done
exit 0
