set -o pipefail
O=gpurun_out/r02_v9; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -rP > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 bash tools/ab_lib.sh default base default base > $O/ab.log 2>&1 || { echo AB FAILED; tail -20 $O/ab.log; exit 1; }
grep "^lib" $O/ab.log
for m in 0 1 2 3; do FISDF_YF_MODE=$m timeout -k 10 120 python tools/ybench.py >> $O/y.log 2>&1 || exit 1; done
cat $O/y.log | grep "y build"
