set -o pipefail
O=gpurun_out/r02_v23; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_isdf.py tests/test_gpu_dist.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/t.log 2>&1 || { echo FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 bash tools/ab_lib.sh default base default base > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
grep "^lib" $O/ab.log | cut -c1-60
