"""Per-kernel duration summary from a rocprofv3 rocpd SQLite database
(rocprofv3's default output format on ROCm 7.2), in the column layout of
rocprofv3's own --stats kernel_stats.csv.

Usage: python scripts/rocpd_stats.py <results.db> [out.csv]
"""
import csv
import sqlite3
import statistics
import sys


def kernel_rows(db):
    c = sqlite3.connect(db)
    tabs = {r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")}
    if "kernels" not in tabs:
        raise SystemExit(f"no kernels view in {db}: {sorted(tabs)}")
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    by = {}
    for n, s, e in c.execute(f"select {name}, start, end from kernels"):
        by.setdefault(n, []).append(e - s)
    return by


def main():
    by = kernel_rows(sys.argv[1])
    total = sum(sum(v) for v in by.values())
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([n, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / total, min(d), max(d),
                    statistics.pstdev(d) if len(d) > 1 else 0.0])


if __name__ == "__main__":
    main()
