set -o pipefail
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_coul.py -k svd > gpurun_out/r04_t3_coul.log 2>&1 || { echo FAIL coul; exit 1; }
timeout -k 10 300 python -u tools/capi_bench.py --steps 10 > gpurun_out/r04_capi_bench.json 2> gpurun_out/r04_capi_bench.err || { echo FAIL capi; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_capi_prof -o capi -- python3 tools/capi_bench.py --steps 5 > gpurun_out/r04_capi_prof.out 2> gpurun_out/r04_capi_prof.err
echo "capi under rocprofv3 rc=$?" >> gpurun_out/r04_capi_prof.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_torch_prof -o torch -- python3 bench.py --steps 5 --no-cpu-baseline --no-isolated > gpurun_out/r04_torch_prof.out 2> gpurun_out/r04_torch_prof.err
echo "torch bench under rocprofv3 rc=$?" >> gpurun_out/r04_torch_prof.out
exit 0
