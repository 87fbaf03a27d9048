"""Per-kernel average of the batch launches from a rocprofv3 kernel trace CSV:
for each kernel, the dispatches with its largest grid (the batch launches;
the latency runs' single-rig launches have smaller grids), averaged.
Usage: kern_avg.py <trace.csv> [max rows] [out.json]  (the JSON maps the kernel
name to its batch-launch average in ms and the number of such launches; bench.py
reads profiles/r03_batch_launch_avg_default.json for its profiled roofline)"""
import json
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
d = collections.defaultdict(list)
for r in rows:
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    d[r["Kernel_Name"]].append((g, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
out = []
for k, v in d.items():
    gmax = max(g for g, _ in v)
    sel = [t for g, t in v if g == gmax]
    out.append((sum(sel) / len(sel), k.split("(")[0][:48], len(sel), len(v)))
out.sort(reverse=True)
for a, k, n, m in out[:top]:
    print(f"{a:9.3f} ms  {k}  ({n} of {m} launches)")
if len(sys.argv) > 3:
    json.dump({k: {"avg_ms": round(a, 4), "launches": n} for a, k, n, m in out}, open(sys.argv[3], "w"), indent=1)
