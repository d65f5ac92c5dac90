set -o pipefail
for i in 1 2; do
timeout -k 10 300 python -u tools/capi_bench.py --steps 10 > gpurun_out/r04_t4_capi_$i.json 2>/dev/null || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/capi_bench.py --steps 10 > gpurun_out/r04_t4_capi_q8_$i.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t4_torch_$i.json 2>/dev/null || exit 1
done
