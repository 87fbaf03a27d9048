"""Summarise a rocprofv3 kernel trace (rocpd sqlite db or kernel_stats.csv) per kernel:
calls, total ms, avg us, share. Usage: prof_summary.py <db-or-csv> [out.md]"""
import csv
import glob
import os
import sqlite3
import sys


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        out = []
        for name, calls, tot, avg, pct in c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"):
            out.append((name, int(calls), float(tot), float(avg), float(pct)))
        return out
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]), float(r["Percentage"])))
    return out


def main():
    p = sys.argv[1]
    if os.path.isdir(p):
        cands = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True) or glob.glob(
            os.path.join(p, "**", "*.db"), recursive=True)
        p = cands[0]
    rows = rows_from(p)
    lines = [f"source: {os.path.basename(p)}", "", "| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for name, calls, tot, avg, pct in rows:
        short = name.split("(")[0].replace("mk::", "")
        lines.append(f"| {short} | {calls} | {tot / 1e6:.3f} | {avg / 1e3:.1f} | {pct:.1f} |")
    txt = "\n".join(lines)
    print(txt)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
