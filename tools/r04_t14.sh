# selection per-pivot latency: where the ~6 us per step goes (timing-only variants, wrong pivots)
set -o pipefail
for e in 0 1 2 3 4 7 0; do
  FISDF_SEL_EXP=$e timeout -k 10 120 python -u tools/select_bench.py --reps 10 2>&1 | grep select || { echo FAIL $e; exit 1; }
done
FISDF_SEL_COOP=0 timeout -k 10 120 python -u tools/select_bench.py --reps 5 2>&1 | grep select
exit 0
