"""Kernel statistics from a rocprofv3 SQLite database (rocpd format).

rocprofv3 >= ROCm 7 writes `<name>_results.db` by default; this turns its
`kernels` view into the same columns `--stats --output-format csv` produces
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev).

    python scripts/rocpd_stats.py gpurun_out/s2/prof/run_results.db > profiles/r01/x.csv
"""
import csv
import math
import sqlite3
import sys


def kernel_stats(db_path):
    con = sqlite3.connect(db_path)
    rows = con.execute("SELECT name, duration FROM kernels").fetchall()
    acc = {}
    for name, dur in rows:
        acc.setdefault(name, []).append(float(dur))
    total = sum(sum(v) for v in acc.values()) or 1.0
    out = []
    for name, v in acc.items():
        n = len(v)
        mean = sum(v) / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        out.append((name, n, sum(v), mean, 100.0 * sum(v) / total, min(v), max(v), sd))
    out.sort(key=lambda r: -r[2])
    return out


def main():
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage",
                "MinNs", "MaxNs", "StdDev"])
    for r in kernel_stats(sys.argv[1]):
        w.writerow([r[0], r[1], int(r[2]), round(r[3], 3), round(r[4], 2), int(r[5]),
                    int(r[6]), round(r[7], 3)])


if __name__ == "__main__":
    main()
