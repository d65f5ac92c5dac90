set -o pipefail
O=gpurun_out/r02_v26; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_isdf.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 -rP --timeout-method thread -k "kmesh_paths or x4_and_y or build_y_qlist or jk_parity_vs or (config_parity_full_size and (c2 or c4 or c5))" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log; grep -E "^c[245]: oracle" $O/tests.log | sed "s/.*ranks/ranks/"
for v in default base; do for m in 0 2; do vv=$v; [ $v = default ] && vv=""; FISDF_LIB_VARIANT=$vv FISDF_YF_MODE=$m timeout -k 10 120 python tools/ybench.py > $O/y.log 2>&1 || exit 1; echo "$v mode $m: $(grep 'y build' $O/y.log | cut -c1-50)"; done; done
timeout -k 10 400 bash tools/ab_lib.sh default base default base > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
grep "^lib" $O/ab.log | cut -c1-200
