#!/bin/bash
# A/B of build variants (fisdf/libfisdf_<v>.so, "" = default) on the C3 bench and the
# GEMM microbenchmark: bash tools/ab_lib.sh v1 v2 ...
set -o pipefail
for v in "$@"; do
  [ "$v" = "default" ] && v=""
  FISDF_LIB_VARIANT=$v timeout -k 10 200 python tools/gemm_bench.py --quick --fx || exit 1
  FISDF_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline > /tmp/abl.json || exit 1
  python - "lib '$v'" /tmp/abl.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(sys.argv[1], d["ms_per_step"], d["roofline"].get("isolated", {}).get("achieved"), d["stages_ms_per_step"])
PY
done
