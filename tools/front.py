"""Critical-path markers of one build from a rocprofv3 kernel trace (round 6): when the
selection, the y build (fused kernel launches), x4, the factor chain, the first TRSM and the last
fit kernel start / end, relative to the build's first kernel.
Usage: python tools/front.py run_kernel_trace.csv [build index, default -2]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = int(sys.argv[2]) if len(sys.argv) > 2 else -2
starts = [i for i, r in enumerate(rows) if "permute_kgm" in r["Kernel_Name"]]
i0 = starts[idx]
i1 = starts[idx + 1] if idx + 1 < len(starts) and idx != -1 else len(rows)
seg = rows[i0:i1]
t0 = int(seg[0]["Start_Timestamp"])


def span(pred):
    s = [r for r in seg if pred(r["Kernel_Name"])]
    if not s:
        return None
    return ((min(int(r["Start_Timestamp"]) for r in s) - t0) / 1e3,
            (max(int(r["End_Timestamp"]) for r in s) - t0) / 1e3, len(s))


marks = {
    "gram (permute+herk)": lambda n: "permute_kgm" in n,
    "selection": lambda n: "pchol_select" in n,
    "y_fused": lambda n: "y_fused_kernel" in n,
    "xt_stream": lambda n: "yf_xt_stream" in n,
    "x4 kmesh": lambda n: "kmesh_y_reg_kernel" in n and "true" in n,
    "chol_diag": lambda n: "chol_diag" in n,
    "trinv": lambda n: "trinv" in n,
    "trsm wide": lambda n: "zgemm_nn_wide" in n,
    "herk reduce": lambda n: "herk_reduce" in n,
    "fft axis0": lambda n: "fft_axis0" in n,
    "fft plane": lambda n: "fft_plane" in n,
}
print(f"build {idx}: {len(seg)} kernels, span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")
for k, p in marks.items():
    v = span(p)
    if v:
        print(f"  {k:22s} {v[0]:10.1f} -> {v[1]:10.1f} us  ({v[2]} launches)")
