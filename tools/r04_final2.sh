# round-end evidence of the final tree (after the folded Gram): smoke, the round profile (bench
# line with CPU baseline, kernel trace, FETCH/WRITE traffic)
set -o pipefail
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/r04_final_smoke.log; exit 1; }
tail -1 gpurun_out/r04_final_smoke.log
bash tools/prof_round.sh r04_prof_v4 || exit 1
exit 0
