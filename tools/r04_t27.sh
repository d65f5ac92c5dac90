# FFT stream priority on the torch path (ROCm 7.0 runtime: least by default) after this round's
# lane speedups: 0 least / 1 default / 2 greatest, three rounds
set -o pipefail
for i in 1 2 3; do
for p in 0 1 2; do
  FISDF_FFT_PRIO=$p timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t27_p${p}_$i.json 2>/dev/null || { echo FAIL $p; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04_t27_p${p}_$i.json').read().strip().splitlines()[-1]); print('prio $p run $i', d['ms_per_step'], 'fft', d['stages_ms_per_step']['fft'], 'trsm', d['stages_ms_per_step']['trsm'])"
done
done
exit 0
