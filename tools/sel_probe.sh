FISDF_SEL_PROF=1 FISDF_SEL_MODE=batch timeout -k 10 120 python -u tools/select_bench.py --cfg c3 --reps 1 2>&1 | grep select
