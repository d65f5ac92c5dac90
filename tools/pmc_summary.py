"""Summarise tools/pmc_gemm.sh passes: per kernel, mean counters and MFMA utilisation."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]; n = n[n.find("::", n.find("namespace)")) + 2:]; k = n[:n.find("(")] + " grid=" + r["Grid_Size"]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    if "zgemm" not in k:
        continue
    m = {n: sum(v) / len(v) for n, v in c.items()}
    line = {n: f"{v:.4g}" for n, v in m.items()}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        # GRBM_GUI_ACTIVE is summed over 8 XCDs; 1024 SIMDs
        line["MfmaUtil%"] = f"{100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.1f}"
    if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
        line["wait_any%"] = f"{100 * m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.1f}"
        line["wait_inst%"] = f"{100 * m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.1f}"
    print(k, line)
