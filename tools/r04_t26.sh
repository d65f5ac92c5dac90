# 1-GPU kernel traces of the final and the pre-change library (3 steps each): where the step's
# critical path runs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default pre; do
  vv=$v; [ "$v" = "default" ] && vv=""
  FISDF_LIB_VARIANT=$vv timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04_t26_$v -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/r04_t26_$v.json 2> gpurun_out/r04_t26_$v.err
  ls gpurun_out/r04_t26_$v/ | grep -q kernel_trace || { echo "no trace $v"; exit 1; }
done
exit 0
