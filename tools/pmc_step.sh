#!/bin/bash
# One rocprofv3 --pmc pass over one C3 bench step for the step-level MFMA-pipe utilisation
# (tools/pmc_step.py).  Usage: bash tools/pmc_step.sh TAG MS_PER_STEP
set -o pipefail
OUT=gpurun_out/${1:-pmcstep}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $OUT/p.log 2>&1
[ -n "$(find $OUT/p -name '*counter_collection.csv')" ] || { echo "pmc pass failed"; tail -20 $OUT/p.log; exit 1; }
python3 tools/pmc_step.py $OUT ${2:-86.3} | tee $OUT/summary.txt
