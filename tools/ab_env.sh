#!/bin/bash
# GPU box: short default bench with and without one environment setting.
# usage: tools/ab_env.sh VAR=value ...   (the plain run goes first)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {
  env $1 timeout -k 10 150 python -u bench.py --steps 5 --warmup 2 --latency-iters 3 --no-cpu --ingest-steps 0 > gpurun_out/abe_$2.json 2> gpurun_out/abe_$2.err || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],d['value'],d['p50_latency_ms'],{k:round(v,2) for k,v in r['stages_ms_isolated'].items() if v>3})" gpurun_out/abe_$2.json $2
}
run "MANTIS_AB_BASE=1" base
i=0; for kv in "$@"; do i=$((i+1)); run "$kv" "v$i:$kv"; done
