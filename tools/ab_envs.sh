#!/bin/bash
# Interleaved A/B of environment settings on the C3 bench: bash tools/ab_envs.sh "A=1 B=2" "" ...
# ("" = defaults); prints ms/step, the dominant-kernel rate and the stage split per setting
set -o pipefail
for e in "$@"; do
  env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline > /tmp/abe.json || exit 1
  python - "$e" /tmp/abe.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"[{sys.argv[1]}]", d["ms_per_step"], d["roofline"]["achieved"], d["stages_ms_per_step"])
PY
done
