"""Reconcile the bench line's HIP-event durations with rocprofv3's on the same
command: per hot kernel, the average launch duration of
each context's stream in the rocprofv3 kernel trace (batch launches only: the
largest grid of that kernel on that stream), the all-context average, and the
bench line's context-0 and all-context event figures printed by that run.

usage: python3 tools/dur_sources.py <rocprof dir> <bench log> > out.txt
"""
import collections
import csv
import json
import os
import sys

HOT = ["k_canny_strip", "k_hyst_rec", "k_score_init", "k_score_pf", "k_score_final"]


def main(d, log):
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    per = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        for w in HOT:
            if ("mk::" + w + "<") in name or ("mk::" + w + "(") in name:
                g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
                per[(w, int(r["Stream_Id"]))].append(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, g))
    line = json.loads([x for x in open(log) if x.startswith("{")][-1])
    roof = line["roofline"]
    print("# per-kernel launch durations (ms) of the batch launches, rocprofv3 kernel trace by stream,")
    print("# against the bench line's HIP events of the same run")
    print("# rocprof dir:", d, " bench log:", log)
    streams = sorted({s for (_, s) in per})
    print("%-14s" % "kernel" + "".join("%9s" % ("s%d" % s) for s in streams) + "%10s" % "all")
    for w in HOT:
        cells, allv = [], []
        for s in streams:
            v = per.get((w, s), [])
            gmax = max((g for _, g in v), default=0)
            big = [t for t, g in v if g == gmax]
            allv += big
            cells.append("%9.2f" % (sum(big) / len(big)) if big else "%9s" % "-")
        print("%-14s" % w + "".join(cells) + ("%10.2f" % (sum(allv) / len(allv)) if allv else ""))
    print("# bench line events: all contexts", roof.get("kernels_ms"), " context 0", roof.get("context0", {}).get("kernels_ms"))
    print("# stream 1 is context 0 (created first); it submits first in every step, so its launches meet")
    print("# fewer of the other contexts' blocks on the CUs than the later streams' launches do")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
