set -o pipefail
O=gpurun_out/r02_v35; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_isdf.py tests/test_gpu_configs.py tests/test_coul.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -rP -k "gamma or si_small or c1 or c5 or Gamma or get_coul or x4_and_y or jk_parity_vs" > $O/t.log 2>&1 || { echo FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log; grep -E "^c[15]: oracle|diamond_szv_gamma: nip|si_small: nip" $O/t.log | sed 's/fit q=.*|dJ/|dJ/' | cut -c1-160
for v in default base default base; do vv=$v; [ $v = default ] && vv=""; FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('$O/c5.json'));print('$v c5', d['ms_per_step'], {k:v for k,v in d['stages_ms_per_step'].items() if k in ('x4','get_k','select','factor')})"; done
