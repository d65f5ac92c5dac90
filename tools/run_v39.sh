set -o pipefail
O=gpurun_out/r02_v39; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -rP > $O/t.log 2>&1 || { echo FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log; grep -E "^c[1-5]: oracle" $O/t.log | cut -c1-160
for cfg in c5 c3; do for v in default base default base; do vv=$v; [ $v = default ] && vv=""; FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline > $O/${cfg}_$v.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('$O/${cfg}_$v.json'));print('$v $cfg', d['ms_per_step'], {k:v for k,v in d['stages_ms_per_step'].items() if k in ('select','factor','y')})"; done; done
