set -o pipefail
OUT=gpurun_out/r06a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -rP > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 60 python -u bench.py --gpus 2 > $OUT/gpus2.out 2>&1; echo "gpus2 rc=$?"; cat $OUT/gpus2.out
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
