"""Summarise a rocprofv3 output directory (rocpd .db or *_kernel_stats.csv)
into a small CSV of per-kernel call counts and durations (microseconds)."""
import csv
import glob
import os
import sqlite3
import sys


def summarise(d, out):
    rows = []
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        with open(stats[0]) as f:
            for r in csv.DictReader(f):
                rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                             float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    elif dbs:
        c = sqlite3.connect(dbs[0])
        for r in c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"):
            rows.append((r[0], int(r[1]), float(r[2]) / 1e3, float(r[3]) / 1e3, float(r[4])))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "average_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], f"{r[2]:.3f}", f"{r[3]:.3f}", f"{r[4]:.2f}"])
    return rows


if __name__ == "__main__":
    for r in summarise(sys.argv[1], sys.argv[2]):
        print(r)
