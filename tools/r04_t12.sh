# A/B: speculative FFTs on/off, emulated 8 ranks and the 1-GPU C3 step (pairs alternate)
set -o pipefail
for i in 1 2; do
for sp in 1 0; do
  FISDF_FIT_SPEC=$sp timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/r04_t12_emu_s${sp}_$i.json 2> gpurun_out/r04_t12_emu_s${sp}_$i.err || { echo FAIL emu; exit 1; }
  FISDF_FIT_SPEC=$sp timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t12_b_s${sp}_$i.json 2>/dev/null || { echo FAIL b; exit 1; }
done
done
exit 0
