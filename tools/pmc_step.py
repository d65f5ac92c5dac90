"""Step-level MFMA-pipe utilisation of the C3 bench from one rocprofv3 --pmc pass
(SQ_INSTS_VALU_MFMA_F64, SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE; tools/pmc_step.sh).
Sums the counters over the dispatches of the first build (from one permute_kgm to the next)
and relates the MFMA-busy time to the unprofiled step time given on the command line:
  python tools/pmc_step.py gpurun_out/<dir> <ms_per_step>"""
import collections
import csv
import glob
import os
import sys

d, ms = sys.argv[1], float(sys.argv[2])
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
disp = collections.OrderedDict()
for r in rows:
    k = int(r["Dispatch_Id"])
    e = disp.setdefault(k, {"name": r["Kernel_Name"], "c": {}})
    e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
items = [disp[k] for k in sorted(disp)]
starts = [i for i, e in enumerate(items) if "permute_kgm" in e["name"]]
seg = items[starts[0]:starts[1]] if len(starts) > 1 else items[starts[0]:]
SIMDS, CLK = 1024, 2.4e9          # MI355X: 256 CUs x 4 SIMDs, 2400 MHz peak engine clock
busy = collections.Counter()
insts = collections.Counter()
for e in seg:
    n = e["name"]
    n = n.replace("fisdf::(anonymous namespace)::", "").replace("void ", "")
    n = n[:n.find("(")] if "(" in n else n
    busy[n] += e["c"].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    insts[n] += e["c"].get("SQ_INSTS_VALU_MFMA_F64", 0.0)
tot_busy = sum(busy.values())
tot_inst = sum(insts.values())
busy_ms = tot_busy / SIMDS / CLK * 1e3
print(f"dispatches in the step: {len(seg)}; FP64 MFMA instructions {tot_inst:.4g} "
      f"({tot_busy / max(tot_inst, 1):.1f} busy cycles each)")
print(f"MFMA-pipe busy time {busy_ms:.1f} ms of a {ms:.1f} ms step: "
      f"{100 * busy_ms / ms:.1f} % of the FP64 MFMA peak over the whole step "
      f"(executed MFMA flop {tot_inst * 2048 / (ms * 1e-3) / 1e12:.1f} TFLOP/s of 78.6)")
for n, b in busy.most_common(8):
    print(f"  {b / SIMDS / CLK * 1e3:7.2f} ms busy  {insts[n]:.3g} MFMA  {n}")
