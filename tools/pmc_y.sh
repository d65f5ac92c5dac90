#!/bin/bash
# PMC passes over the fused-y microbenchmark (tools/ybench.py): wait / issue breakdown of
# y_fused_kernel, one rocprofv3 run per counter set.  Usage: bash tools/pmc_y.sh TAG [YF_MODE]
set -o pipefail
OUT=gpurun_out/${1:-pmcy}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  FISDF_YF_MODE=${2:-0} timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 tools/ybench.py --reps 2 > $OUT/p$i.log 2>&1
  [ -n "$(find $OUT/p$i -name '*counter_collection.csv')" ] || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import collections, csv, glob, os, sys
d = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if "y_fused" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
for k in sorted(m):
    print(f"{k:28s} {m[k]:.4g}")
wc = m.get("SQ_WAVE_CYCLES", 1)
print("per wave-cycle: wait_any %.2f wait_inst %.2f active_any %.2f active_valu %.2f" % (
    m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
    m.get("SQ_ACTIVE_INST_VALU", 0) / wc))
if "GRBM_GUI_ACTIVE" in m:
    print("MFMA util %.1f %%" % (100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)))
PY
