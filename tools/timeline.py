"""Kernel timeline of one bench step from a rocprofv3 --kernel-trace CSV.

Usage: python tools/timeline.py run_kernel_trace.csv [--step N] [--from NAME] [--count K]
Prints kernel start (us, relative), duration, the idle gap before it and the stream/queue, for
the launches of step N (steps are split at each zgemm<...,true,...> selection Gram: the first
kernel of a build)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step", type=int, default=-1, help="build index (default: last)")
    ap.add_argument("--count", type=int, default=120)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--marker", default="permute_kgm", help="kernel name that starts a build")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if not starts:
        raise SystemExit("marker not found")
    i0 = starts[a.step]
    i1 = starts[a.step + 1] if a.step + 1 < len(starts) and a.step != -1 else len(rows)
    seg = rows[i0:i1]
    t0 = int(seg[0]["Start_Timestamp"])
    end = t0
    print(f"{len(seg)} kernels, span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")
    for r in seg[a.skip:a.skip + a.count]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - end) / 1e3
        end = max(end, e)
        name = r["Kernel_Name"].replace("fisdf::(anonymous namespace)::", "")[:70]
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f} gap {gap:7.1f} q{r.get('Queue_Id', '?'):>3} {name}")


if __name__ == "__main__":
    main()
