set -o pipefail
O=gpurun_out/r02_v36; mkdir -p $O
FISDF_SEL_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_isdf.py -m gpu -x -q -s --timeout 200 --timeout-method thread -k "selection_paths_agree" > $O/sel.log 2>&1 || { echo FAILED sel; tail -30 $O/sel.log; exit 1; }
grep -c "K=20" $O/sel.log; grep "dpstrf:" $O/sel.log; tail -1 $O/sel.log
FISDF_SEL_DEBUG=1 timeout -k 10 300 python -u -c "
import bench, sys
" > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_selection.py tests/test_gpu_configs.py -m gpu -x -q --timeout 500 --timeout-method thread -rP -k "c5 or c3 or c1" > $O/t.log 2>&1 || { echo FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log; grep -E "^c[135]: " $O/t.log | cut -c1-220
for v in default base default base; do vv=$v; [ $v = default ] && vv=""; FISDF_SEL_DEBUG=1 FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5_$v.json 2>$O/c5_$v.err || exit 1; python -c "import json;d=json.load(open('$O/c5_$v.json'));print('$v c5', d['ms_per_step'], {k:v for k,v in d['stages_ms_per_step'].items() if k in ('select','factor')})"; done
grep -m1 cooperative $O/c5_default.err
