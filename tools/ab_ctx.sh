#!/bin/bash
# GPU box: default bench at several contexts x rigs (A/B/A/B order)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --latency-iters 1 --no-cpu --ingest-steps 0 $1 > gpurun_out/abc.json 2> gpurun_out/abc.err || { tail -3 gpurun_out/abc.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step'])" gpurun_out/abc.json "$1"
}
for rep in 1 2; do
  run "--contexts 6 --rigs 6144"
  run "--contexts 8 --rigs 6144"
  run "--contexts 7 --rigs 7168"
  run "--contexts 5 --rigs 6144"
done
