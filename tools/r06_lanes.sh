#!/bin/bash
# Fit-lane serialisation A/B: C3 bench (3 steps) under launch / stream variants,
# each line: variant, ms/step, TRSM and HERK average launch (ms; ~0.95 / 0.92 = lanes serialised,
# ~1.74 / 1.23 = overlapped).  Then the group crash with the cooperative-launch mutex off under
# the runtime log (how many cooperative queues the rank threads create).
# Usage: bash tools/r06_lanes.sh TAG [ab2]
set -o pipefail
TAG=${1:-r06_lanes}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env FISDF_NOOP=1 "$@" timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > $OUT/$name.json 2> $OUT/$name.err || { echo "$name FAILED"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); s=d['stages_ms_per_step']; print('$name', d['ms_per_step'], round(d['roofline']['avg_launch_ms'],3), round(d['roofline_secondary']['avg_launch_ms'],3), 'sel', s['select'], 'y', s['y'])"
}
if [ "$2" = "ab6" ]; then
run ys && \
run ys_g242 FISDF_SEL_WGS=242 && \
run ys_g176 FISDF_SEL_WGS=176 && \
run ys_r32 FISDF_Y_STREAM_ROWS=32 && \
run ys_b && \
run ys_g242_b FISDF_SEL_WGS=242 && \
run ys_r32_b FISDF_Y_STREAM_ROWS=32 || exit 1
exit 0
fi
if [ "$2" = "ab5" ]; then
run base && \
run aux0 FISDF_Y_STREAM_AUX=0 && \
run aux0_fft64 FISDF_Y_STREAM_AUX=0 FISDF_FFT_CUS=64 && \
run aux0_fft128 FISDF_Y_STREAM_AUX=0 FISDF_FFT_CUS=128 && \
run aux0_fft192 FISDF_Y_STREAM_AUX=0 FISDF_FFT_CUS=192 && \
run base_b && \
run aux0_fft128_b FISDF_Y_STREAM_AUX=0 FISDF_FFT_CUS=128 && \
run aux0_b FISDF_Y_STREAM_AUX=0 || exit 1
exit 0
fi
if [ "$2" = "ab4" ]; then
run coop_ys FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 && \
run plain_ys FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 && \
run coop FISDF_Y_STREAM=0 && \
run plain FISDF_Y_STREAM=0 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 && \
run coop_ys_b FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 && \
run plain_ys_b FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 && \
run coop_b FISDF_Y_STREAM=0 && \
run plain_b FISDF_Y_STREAM=0 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 || exit 1
FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-isolated --steps 3 --warmup 1 > $OUT/prof_bench.json 2> $OUT/prof.err
echo "profiled plain_ys rc=$?"
exit 0
fi
if [ "$2" = "ab3" ]; then
run base FISDF_Y_STREAM=0 && \
run ys2 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 && \
run ys2_g242 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 FISDF_SEL_WGS=242 && \
run ys0_g242 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=0 FISDF_SEL_WGS=242 && \
run base_g242 FISDF_Y_STREAM=0 FISDF_SEL_WGS=242 && \
run base_b FISDF_Y_STREAM=0 && \
run ys2_g242_b FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 FISDF_SEL_WGS=242 && \
run ys2_b FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 || exit 1
for v in "0 128" "1 128" "1 242"; do set -- $v
  FISDF_Y_STREAM=$1 FISDF_SEL_WGS=$2 timeout -k 10 400 python -u bench.py --emulate-ranks 8 --steps 5 --warmup 2 > $OUT/emu8_ys$1_g$2.json 2> $OUT/emu8_ys$1_g$2.err || { echo "EMU $v FAILED"; tail -20 $OUT/emu8_ys$1_g$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/emu8_ys$1_g$2.json')); print('emu8 ys=$1 g=$2 max', d['max_rank_ms'], [r['ms_per_step'] for r in d['ranks']])"
done
exit 0
fi
if [ "$2" = "ab2" ]; then
run base FISDF_Y_STREAM=0 && \
run ys_aux0 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=0 && \
run ys_aux1 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=1 && \
run ys_aux2 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 && \
run plain_pad1 FISDF_Y_STREAM=0 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 && \
run base_b FISDF_Y_STREAM=0 && \
run ys_aux1_b FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=1 && \
run plain_pad1_b FISDF_Y_STREAM=0 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 && \
run ys_plain_pad1 FISDF_Y_STREAM=1 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 || exit 1
exit 0
fi
run base FISDF_Y_STREAM=0 && \
run ys_aux1 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=1 && \
run ys_aux2 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=2 && \
run ys_aux0 FISDF_Y_STREAM=1 FISDF_Y_STREAM_AUX=0 && \
run plain FISDF_Y_STREAM=0 FISDF_COOP_LAUNCH=0 && \
run plain_pad1 FISDF_Y_STREAM=0 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=1 && \
run plain_pad2 FISDF_Y_STREAM=0 FISDF_COOP_LAUNCH=0 FISDF_PAD_QUEUES=2 || exit 1
D=$(mktemp -d)
FISDF_COOP_MUTEX=0 AMD_LOG_LEVEL=3 timeout -k 10 240 python3 -u tests/capi_shard_worker.py toy331_fr 0 3 $D group > $OUT/group_m0.out 2> $OUT/group_m0.amdlog
echo "group mutex=0 rc=$? cooperative queues created: $(grep -c 'cooperative: 1' $OUT/group_m0.amdlog)"
grep -E "SWq|cooperative queue" $OUT/group_m0.amdlog | cut -c1-300 > $OUT/group_m0_queues.txt
gzip -f $OUT/group_m0.amdlog
rm -rf $D
exit 0
