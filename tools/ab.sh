#!/bin/bash
# One parameterised GPU session (replaces round 4's one-off tools/r04_t*.sh drivers):
#   bash tools/ab.sh TAG [-t "PYTEST ARGS"] [-r REPS] [-e] [-1] [-p] [VARIANT ...]
#   -t  run this pytest selection first (stops on failure)
#   -r  interleaved repetitions of the variant list (default 2)
#   -e  per variant: bench.py --emulate-ranks 8 (the per-rank step of an 8-way build)
#   -1  per variant: the 1-GPU C3 step (bench.py --no-cpu-baseline --no-isolated; default when
#       neither -e nor -1 is given)
#   -p  afterwards: the round profile (tools/prof_round.sh TAG_prof)
#   VARIANT: "default", an environment assignment list "FISDF_A=1,FISDF_B=0", or "lib:NAME"
#            (loads fisdf/libfisdf_NAME.so, built by tools/build_variant.sh)
# Output under gpurun_out/TAG/: one JSON per run, summary lines on stdout.  Every GPU step runs
# under its own timeout; the first failure ends the session.
set -o pipefail
TAG=$1; shift
TESTS=""; REPS=2; EMU=0; ONE=0; PROF=0
while getopts "t:r:e1p" o; do
  case $o in
    t) TESTS=$OPTARG ;; r) REPS=$OPTARG ;; e) EMU=1 ;; 1) ONE=1 ;; p) PROF=1 ;;
    *) echo "bad option"; exit 2 ;;
  esac
done
shift $((OPTIND - 1))
[ $# -eq 0 ] && set -- default
[ $EMU -eq 0 ] && ONE=1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS -x -v -s --timeout 600 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|ERROR|^E " $OUT/tests.log | tail -30; tail -5 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
run_variant() {  # $1 variant, $2 rep
  local v=$1 i=$2 name envs=() lib=""
  name=$(echo "$v" | tr ',=:' '_.-')
  case $v in
    default) ;;
    lib:*) lib=${v#lib:} ;;
    *) IFS=',' read -ra envs <<< "$v" ;;
  esac
  if [ $ONE -eq 1 ]; then
    env "${envs[@]}" FISDF_LIB_VARIANT=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline \
      --no-isolated $BENCH_ARGS > $OUT/b_${name}_$i.json 2> $OUT/b_${name}_$i.err \
      || { echo "BENCH FAILED ($v)"; tail -20 $OUT/b_${name}_$i.err; return 1; }
    python3 - $OUT/b_${name}_$i.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d.get("stages_ms_per_step", {})
print("1gpu", sys.argv[2], d["ms_per_step"], {k: s[k] for k in ("select", "y", "factor", "fft", "trsm", "herk") if k in s})
PY
  fi
  if [ $EMU -eq 1 ]; then
    env "${envs[@]}" FISDF_LIB_VARIANT=$lib timeout -k 10 400 python -u bench.py --emulate-ranks 8 \
      --steps 10 --warmup 2 > $OUT/e_${name}_$i.json 2> $OUT/e_${name}_$i.err \
      || { echo "EMULATE FAILED ($v)"; tail -20 $OUT/e_${name}_$i.err; return 1; }
    python3 - $OUT/e_${name}_$i.json "$v" <<'PY'
import json, sys
e = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("emu8", sys.argv[2], "max", e["max_rank_ms"], [round(x["ms_per_step"], 2) for x in e["ranks"]])
PY
  fi
}
for i in $(seq 1 $REPS); do
  for v in "$@"; do
    run_variant "$v" $i || exit 1
  done
done
if [ $PROF -eq 1 ]; then
  bash tools/prof_round.sh ${TAG}_prof || exit 1
fi
exit 0
