# timing-only what-if variants (wrong numerics): how much of the C3 step each piece holds
set -o pipefail
for i in 1 2; do
for v in default nored norealtrsm nofft noy; do
  vv=$v; [ "$v" = "default" ] && vv=""
  FISDF_LIB_VARIANT=$vv timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-isolated > gpurun_out/r04_wi_${v}_$i.json 2>/dev/null || echo "fail $v"
done
done
exit 0
