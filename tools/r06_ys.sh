#!/bin/bash
# Streamed y (y behind the selection): parity tests (1-GPU streamed vs unstreamed, the k-sharded
# mirror through gloo ranks and the emulated 8-rank C3), then C3 bench streamed / unstreamed,
# the emulated 8-rank step both ways, then the crash + queue-mapping probe.
# Usage: bash tools/r06_ys.sh TAG [noprobe]
set -o pipefail
TAG=${1:-r06_ys}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_isdf.py tests/test_gpu_dist.py tests/test_gpu_shard_full.py -k "streamed_y or dist or c3" -x -v --timeout 600 --timeout-method thread -rP > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "PASSED|FAILED|ERROR|^E |streamed" $OUT/t.log | tail -40; exit 1; }
grep -E "streamed|passed|failed" $OUT/t.log | tail -12
for ab in 1 0 1 0; do
  FISDF_Y_STREAM=$ab timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-isolated > $OUT/bench_ys$ab.json 2> $OUT/bench_ys$ab.err || { echo "BENCH ys=$ab FAILED"; tail -20 $OUT/bench_ys$ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_ys$ab.json')); print('ys=$ab', d['ms_per_step'], {k: v for k, v in d['stages_ms_per_step'].items() if k in ('select','x4','y','factor')})"
done
for ab in 1 0; do
  FISDF_Y_STREAM=$ab timeout -k 10 400 python -u bench.py --emulate-ranks 8 --steps 5 --warmup 2 > $OUT/emu8_ys$ab.json 2> $OUT/emu8_ys$ab.err || { echo "EMU ys=$ab FAILED"; tail -20 $OUT/emu8_ys$ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/emu8_ys$ab.json')); print('emu8 ys=$ab max', d['max_rank_ms'], [r['ms_per_step'] for r in d['ranks']])"
done
[ "$2" = "noprobe" ] && exit 0
bash tools/crash_probe.sh ${TAG}_probe
