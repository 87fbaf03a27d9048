#!/bin/bash
# GPU box: instruction-cache counters of every kernel under the default
# 6-context command (one --pmc pass: SQC_ICACHE_HITS / _MISSES beside the SQ
# wave-cycle and instruction-wait counters), summarised per kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/icache; mkdir -p $O; export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU -f csv -d "$R/$O/p" -o run -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 --latency-iters 1 --ingest-steps 0 $BARGS > "$R/$O/p.log" 2>&1) || { echo pmc failed; tail -5 $O/p.log; exit 1; }
python3 - "$O/p" <<'P'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
rows = []
for k, d in acc.items():
    h, m = d.get("SQC_ICACHE_HITS", 0), d.get("SQC_ICACHE_MISSES", 0)
    wc = d.get("SQ_WAVE_CYCLES", 0)
    rows.append((wc, k, h, m, m / max(1, h + m), d.get("SQ_WAIT_INST_ANY", 0) / max(1, wc)))
for wc, k, h, m, mr, wi in sorted(rows, reverse=True)[:20]:
    print(f"{k:40s} icache miss rate {mr:.4f} (misses {m:.3g}) wait_inst/wave_cycles {wi:.3f} wave_cycles {wc:.3g}")
P
