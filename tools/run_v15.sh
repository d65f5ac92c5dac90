set -o pipefail
O=gpurun_out/r02_v15; mkdir -p $O
FISDF_YF_GPAIR=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_isdf.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kmesh_paths or x4_and_y" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for g in 1 2 4 8; do for m in 0 2; do FISDF_YF_MODE=$m FISDF_YF_GPAIR=$g timeout -k 10 120 python tools/ybench.py > $O/y_${g}_$m.log 2>&1 || exit 1; echo "gpair $g mode $m: $(grep 'y build' $O/y_${g}_$m.log)"; done; done
