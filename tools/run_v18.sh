set -o pipefail
O=gpurun_out/r02_v18; mkdir -p $O
for e in "FISDF_WPP_TRI=1 FISDF_FACTOR_KEEP=1" "FISDF_WPP_TRI=0 FISDF_FACTOR_KEEP=1" "FISDF_WPP_TRI=1 FISDF_FACTOR_KEEP=0" "FISDF_WPP_TRI=0 FISDF_FACTOR_KEEP=0"; do
  env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_isdf.py tests/test_gpu_configs.py -m gpu -q --timeout 250 --timeout-method thread -rP -k "(jk_parity_vs_oracle and toy331_fr) or (config_parity_full_size and c5)" > $O/t.log 2>&1 || { echo FAILED $e; tail -30 $O/t.log; exit 1; }
  echo "[$e]"; grep -E "toy331_fr: nip|^c5: oracle|^c5: q" $O/t.log | cut -c1-40,150-230
done
