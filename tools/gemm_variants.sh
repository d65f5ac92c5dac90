set -o pipefail
for v in "" bk4n4 bk4n6 bk4n8; do
  echo "== variant '$v'"
  FISDF_LIB_VARIANT=$v timeout -k 10 120 python tools/gemm_bench.py || exit 1
done
for v in "" bk4n6 bk4n8; do
  FISDF_LIB_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > /tmp/b_$v.json || exit 1
  python -c "import json,sys;d=json.load(open('/tmp/b_$v.json'));print('bench $v',d['ms_per_step'],d['roofline']['isolated'],d['stages_ms_per_step'])"
done
