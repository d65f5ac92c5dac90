set -o pipefail
O=gpurun_out/r02_v19; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_isdf.py tests/test_gpu_configs.py tests/test_gpu_kernels.py -m gpu -q --timeout 400 --timeout-method thread -rP -k "(jk_parity_vs_oracle and toy331_fr) or config_parity_full_size or min_norm or unpivoted" > $O/t.log 2>&1 || { echo FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
grep -E "toy331_fr: nip|^c[1-5]: oracle|^c[1-5]: q" $O/t.log | cut -c1-40,100-230
timeout -k 10 400 bash tools/ab_lib.sh default base default base > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
grep "^lib" $O/ab.log | cut -c1-200
