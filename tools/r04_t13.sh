# factor chain at the 8-rank batch (5 q) alone: wall time and per-kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/factor_bench.py --batches 5 4 36 --reps 10 > gpurun_out/r04_t13_factor.txt 2>&1 || { echo FAIL; cat gpurun_out/r04_t13_factor.txt; exit 1; }
cat gpurun_out/r04_t13_factor.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_t13_prof -o fac -- python -u tools/factor_bench.py --batches 5 --reps 10 > gpurun_out/r04_t13_prof.log 2>&1 || echo "prof rc=$?"
exit 0
