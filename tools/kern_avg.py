"""Per-kernel average of the batch launches (the 4 longest dispatches of each
kernel) from a rocprofv3 kernel trace CSV. Usage: kern_avg.py <trace.csv> [n]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keep = int(sys.argv[2]) if len(sys.argv) > 2 else 4
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = sorted(((sum(sorted(v)[-keep:]) / min(keep, len(v)), k.split("(")[0][:48], len(v)) for k, v in d.items()),
             reverse=True)
for a, k, n in out[:40]:
    print(f"{a:9.3f} ms  {k}  ({n})")
