"""Per-launch HBM traffic of the roofline kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
(MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced streaming reads -> doubled here).  Prints one JSON object.
  python tools/traffic.py gpurun_out/<tag>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {  # label: kernel-name substring (the hot launches: the grid carrying the most bytes)
    "herk": "zgemm_glds_kernel<0, 3, true, 0, 3, true>",    # Coulomb HERK, pipelined 3M loop
    "trsm_gemm": "zgemm_nn_wide_kernel<4, 3>",             # lower-triangular GEMM U = L^-1 Yhat
    "fft_plane": "fft_plane_reg<36>",
    "fft_axis0": "fft_axis0_reg<36>",
    "y_fused": "y_fused_kernel<4, 4, 4>",
}


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = list(csv.DictReader(open(f[0]))) if f else []
    out = defaultdict(list)
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        out[r["Kernel_Name"]].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    return out


def main():
    d = sys.argv[1]
    fetch = load(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = load(os.path.join(d, "write"), "WRITE_SIZE")
    res = {}
    for label, sub in KERNELS.items():
        fk = [v for k, v in fetch.items() if sub in k]
        wk = [v for k, v in write.items() if sub in k]
        if not fk or not wk:
            continue
        fl, wl = fk[0], wk[0]
        # the hot-path launches: the grid size that carries the most counted bytes (for the
        # HERK: the per-q fit launches, not the selection Gram or the Im-correction HERKs)
        from collections import Counter
        tot = Counter()
        for g, v in fl:
            tot[g] += v
        gmax = tot.most_common(1)[0][0]
        fsel = [v for g, v in fl if g == gmax]
        wsel = [v for g, v in wl if g == gmax]
        fb = 2.0 * 1024 * sum(fsel) / len(fsel)   # gfx950: FETCH_SIZE counts half (x2), KB
        wb = 1024 * sum(wsel) / len(wsel)
        res[label] = {"launches": len(fsel), "grid": gmax, "fetch_bytes": fb, "write_bytes": wb,
                      "hbm_bytes_per_launch": fb + wb}
    res["source"] = os.path.basename(os.path.normpath(d))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
