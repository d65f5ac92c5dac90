set -o pipefail
O=gpurun_out/r02_v12; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_isdf.py tests/test_gpu_selection.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kmesh_paths or x4_and_y or build_y_qlist or jk_parity_vs or selection" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in 0 1 2; do FISDF_YF_MODE=$m timeout -k 10 120 python tools/ybench.py > $O/y_$m.log 2>&1 || exit 1; echo "mode $m: $(grep 'y build' $O/y_$m.log)"; done
timeout -k 10 300 bash tools/ab_envs.sh "" "" > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
cat $O/ab.log | grep "^\["
