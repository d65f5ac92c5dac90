set -o pipefail
O=gpurun_out/r02_v10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_isdf.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kmesh_paths or x4_and_y or build_y_qlist or jk_parity_vs" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for g in 0 4 6 8 12 19; do FISDF_YF_IGRP=$g timeout -k 10 120 python tools/ybench.py > $O/y_$g.log 2>&1 || exit 1; echo "igrp $g: $(grep 'y build' $O/y_$g.log)"; done
for g in 0 8; do FISDF_YF_MODE=2 FISDF_YF_IGRP=$g timeout -k 10 120 python tools/ybench.py > $O/ym2_$g.log 2>&1 || exit 1; echo "mode2 igrp $g: $(grep 'y build' $O/ym2_$g.log)"; done
timeout -k 10 300 bash tools/ab_envs.sh "" "FISDF_YF_IGRP=0" "" "FISDF_YF_IGRP=0" > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
cat $O/ab.log | grep "^\["
