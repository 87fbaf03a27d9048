#!/bin/bash
# SQ counters of the RPP kernels (GPU box): tools/pmc_rpp.sh TAG [size]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=$1; N=${2:-600}
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -f csv -d "$R/gpurun_out/pmc_$TAG" -o run -- python3 "$R/tools/bench_rpp.py" $N > "$R/gpurun_out/pmc_$TAG.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_$TAG.log"; exit 1; }
python3 - "$R/gpurun_out/pmc_$TAG" <<'P'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    if "objpose" not in k and "s1b" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    w = max(d["SQ_WAVES"], 1)
    print(k, {c: round(v / w, 1) for c, v in sorted(d.items())}, "waves", w)
P
