set -o pipefail
for i in 1 2; do
for p in 0 1 2; do
FISDF_FFT_PRIO=$p timeout -k 10 300 python -u tools/capi_bench.py --steps 10 > gpurun_out/r04_t5_capi_p${p}_$i.json 2>/dev/null || exit 1
FISDF_FFT_PRIO=$p timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t5_torch_p${p}_$i.json 2>/dev/null || exit 1
done
done
