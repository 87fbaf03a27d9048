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
    # per-batch averages: dispatches at each kernel's largest grid (the batch
    # launches of the timed region and warmup; the small ones are the p50
    # single-rig latency calls), comparable with bench.py's avg_launch_ms
    tr = glob.glob(os.path.join(os.path.dirname(p), "**", "*kernel_trace.csv"), recursive=True)
    if tr:
        per = {}
        for r in csv.DictReader(open(tr[0])):
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per.setdefault(r["Kernel_Name"].split("(")[0].replace("mk::", ""), []).append((g, d))
        lines += ["", "Batch launches only (each kernel's largest grid):", "",
                  "| kernel | batch launches | avg us | min us | max us |", "|---|---:|---:|---:|---:|"]
        rows2 = []
        for k, v in per.items():
            gmax = max(g for g, _ in v)
            ds = [d for g, d in v if g == gmax]
            rows2.append((sum(ds) / len(ds), k, ds))
        for avg, k, ds in sorted(rows2, reverse=True):
            lines.append(f"| {k} | {len(ds)} | {avg:.1f} | {min(ds):.1f} | {max(ds):.1f} |")
    txt = "\n".join(lines)
    print(txt)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
