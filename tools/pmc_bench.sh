#!/bin/bash
# SQ counters per kernel for a small single-context bench run (GPU box):
# tools/pmc_bench.sh TAG "COUNTERS..." [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=$1; CNT=$2; shift 2
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CNT -f csv -d "$R/gpurun_out/pmc_$TAG" -o run -- python3 "$R/bench.py" --no-cpu --rigs 64 --contexts 1 --steps 2 --warmup 1 --latency-iters 1 "$@" > "$R/gpurun_out/pmc_$TAG.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_$TAG.log"; exit 1; }
python3 - "$R/gpurun_out/pmc_$TAG" <<'P'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("mk::", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, d in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    n = len(disp[k])
    print(f"{k:28s} dispatches {n:3d} " + " ".join(f"{c}={v / n:.4g}" for c, v in sorted(d.items())))
P
