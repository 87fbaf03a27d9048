#!/bin/bash
# GPU box: short default bench under each value of one environment variable.
# usage: tools/sweep_env.sh VAR v1 v2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
VAR=$1; shift
for v in "$@"; do
  env "$VAR=$v" timeout -k 10 150 python -u bench.py --steps 5 --warmup 2 --latency-iters 1 --no-cpu --ingest-steps 0 > gpurun_out/sw_$v.json 2> gpurun_out/sw_$v.err || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],round(d['roofline']['stages_ms']['rpp_first'],1),round(d['roofline']['stages_ms']['rpp_cand'],1))" gpurun_out/sw_$v.json "$VAR=$v"
done
