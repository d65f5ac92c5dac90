#!/bin/bash
# A/B of one environment knob on the C3 bench: bash tools/ab_env.sh VAR v1 v2 ...
# prints ms/step, the HERK roofline and the stage split per value
set -o pipefail
VAR=$1
shift
for v in "$@"; do
  env "$VAR=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline > /tmp/ab_$v.json || exit 1
  python - "$v" /tmp/ab_$v.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(sys.argv[1], d["ms_per_step"], d["roofline"]["achieved"], d["stages_ms_per_step"])
PY
done
