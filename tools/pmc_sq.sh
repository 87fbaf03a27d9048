#!/bin/bash
# SQ issue/stall breakdown per kernel (GPU box): one --pmc pass of <= 8 SQ
# counters over a short bench run; writes gpurun_out/pmc_${PMC_TAG:-sq}/ and prints
# per-kernel averages. Usage: bash tools/pmc_sq.sh [COUNTERS...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
C=${*:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU}
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -f csv -d "$R/gpurun_out/pmc_${PMC_TAG:-sq}" -o run -- python3 "$R/bench.py" --no-cpu --rigs 512 --contexts 1 --steps 2 --warmup 1 --latency-iters 1 --ingest-steps 0 > "$R/gpurun_out/pmc_${PMC_TAG:-sq}.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_${PMC_TAG:-sq}.log"; exit 1; }
python3 - "$R/gpurun_out" "${PMC_TAG:-sq}" <<'P'
import csv, glob, sys, collections
f = glob.glob(f"{sys.argv[1]}/pmc_{sys.argv[2]}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    print(k[:40], " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
P
