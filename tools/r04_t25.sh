# 1-GPU A/B on one box: the working library vs libfisdf_pre.so (tools/build_base.sh REV pre)
# (DFT x4, one-call W_s blocks, the faster HERK reduce), three alternating pairs
set -o pipefail
for i in 1 2 3; do
for v in default pre; do
  vv=$v; [ "$v" = "default" ] && vv=""
  FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_t25_${v}_$i.json 2>/dev/null || { echo FAIL $v; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04_t25_${v}_$i.json').read().strip().splitlines()[-1]); print('$v run $i', d['ms_per_step'], 'x4', d['stages_ms_per_step']['x4'], 'herk', d['stages_ms_per_step']['herk'])"
done
done
exit 0
