"""Occupancy of the GPU timeline in a rocprofv3 kernel trace (measurement
tool): over the window of the last N dispatches of the largest-grid k_canny
(one per context and step), the union of busy time, the mean number of
kernels in flight, and per kernel family the summed duration and the time it
ran with no other kernel beside it.

    python tools/trace_overlap.py gpurun_out/prof_TAG [steps]
"""
import collections
import csv
import glob
import sys


def main(d, steps=None):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    ev = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        name = name.split("<")[0]
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, g))
    ev.sort()
    canny = [e for e in ev if e[2] in ("mk::k_canny", "mk::k_canny_strip")]
    gmax = max(e[3] for e in canny)
    big = [e for e in canny if e[3] == gmax]
    k = steps if steps else max(1, len(big) // 2)
    # window: from the k-th last big Canny before the isolated step (bench.py
    # runs context 0 alone for one step after the timed ones: its Canny is the
    # last big one) to that step's start, so the isolated step and the latency
    # calls after it do not count as idle time of the timed steps
    t0 = big[-k - 1][0] if len(big) > k else big[0][0]
    t1 = big[-1][0]
    win = [e for e in ev if e[1] > t0 and e[0] < t1]
    # sweep line
    pts = []
    for s, e, n, _ in win:
        s = max(s, t0)
        e = min(e, t1)
        pts.append((s, 1, n))
        pts.append((e, -1, n))
    pts.sort(key=lambda p: (p[0], p[1]))
    active = collections.Counter()
    busy = 0
    last = t0
    area = 0
    alone = collections.Counter()
    for tt, dlt, n in pts:
        dt = tt - last
        tot = sum(active.values())
        if tot > 0:
            busy += dt
            area += dt * tot
            if tot == 1:
                (only,) = [x for x, c in active.items() if c]
                alone[only] += dt
        active[n] += dlt
        if active[n] == 0:
            del active[n]
        last = tt
    span = t1 - t0
    dur = collections.Counter()
    cnt = collections.Counter()
    for s, e, n, _ in win:
        dur[n] += min(e, t1) - max(s, t0)
        cnt[n] += 1
    print(f"window {span / 1e6:.1f} ms from the last {k} big k_canny dispatches; busy {busy / span:.3f}, "
          f"mean kernels in flight {area / max(busy, 1):.2f}")
    print(f"{'kernel':34s} {'n':>6s} {'sum ms':>9s} {'alone ms':>9s}")
    for n, v in dur.most_common(30):
        print(f"{n:34s} {cnt[n]:6d} {v / 1e6:9.2f} {alone[n] / 1e6:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
