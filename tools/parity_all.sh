#!/bin/bash
# Full-size parity (GPU vs the gelsy oracle on the GPU's points) on every bench config.
set -o pipefail
mkdir -p gpurun_out/parity
for c in c2 c5 c4 c3; do
  timeout -k 10 600 python -u tests/parity_full.py --config $c > gpurun_out/parity/$c.log 2>&1 || { echo "PARITY $c FAILED"; tail -20 gpurun_out/parity/$c.log; exit 1; }
  tail -1 gpurun_out/parity/$c.log
done
