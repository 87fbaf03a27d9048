#!/bin/bash
# GPU box: config-5 (dense hypothesis grid) and config-2 bench legs for the
# in-tree library and an alternative build, alternating twice.
# usage: tools/ab_c5.sh lib.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {  # tag lib config
  MANTIS_AMD_LIB=$2 timeout -k 10 300 python -u bench.py --config $3 --steps 5 --warmup 2 --no-cpu --latency-iters 5 > gpurun_out/abc_$1_c$3.json 2> gpurun_out/abc_$1_c$3.err || { tail -5 gpurun_out/abc_$1_c$3.err; return 1; }
  python3 - gpurun_out/abc_$1_c$3.json $1 $3 <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "config", sys.argv[3], d["metric"], d["value"], d["unit"], "p50", d.get("p50_latency_ms"), flush=True)
P
}
for rep in 1 2; do
  run base "$R/mantis_amd/libmantis_amd.so" 5 || exit 1
  run alt "$R/$1" 5 || exit 1
done
run base "$R/mantis_amd/libmantis_amd.so" 2 || exit 1
