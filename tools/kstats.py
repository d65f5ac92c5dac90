"""Kernel statistics (name, calls, total/avg ms, %) from a rocprofv3 .db (sqlite) or
kernel_stats.csv.  Usage: python tools/kstats.py <results.db|kernel_stats.csv> [out.csv]"""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start) from kernels "
                     "group by name order by sum(end-start) desc").fetchall()
    return [(n, k, tot / 1e6, avg / 1e6) for n, k, tot, avg in rows]


def main():
    src = sys.argv[1]
    rows = from_db(src)
    total = sum(r[2] for r in rows)
    out = [("Name", "Calls", "TotalDurationMs", "AverageMs", "Percentage")]
    out += [(n, k, round(t, 4), round(a, 5), round(100 * t / total, 2)) for n, k, t, a in rows]
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            csv.writer(f).writerows(out)
    for r in out[:30]:
        print(f"{str(r[0])[:90]:90s} {r[1]:>6} {r[2]:>10} {r[3]:>10} {r[4]:>6}")


if __name__ == "__main__":
    main()
