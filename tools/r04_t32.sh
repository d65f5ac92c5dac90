# selection kernel phase timing (FISDF_SEL_PROF), then the round-end smoke + profile
set -o pipefail
FISDF_SEL_PROF=1 timeout -k 10 120 python -u tools/select_bench.py --reps 3 2>&1 | grep "select" || { echo PROBE FAILED; exit 1; }
bash tools/r04_final2.sh
