#!/bin/bash
# GPU box: default bench (short) against alternative builds of the library.
# usage: tools/ab_libs.sh lib1.so lib2.so ...  (the in-tree library runs first)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {
  MANTIS_AMD_LIB=$1 timeout -k 10 150 python -u bench.py --steps 5 --warmup 2 --latency-iters 1 --no-cpu --ingest-steps 0 > gpurun_out/ab_$2.json 2> gpurun_out/ab_$2.err || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],d['value'],{k:round(v,2) for k,v in r['stages_ms_isolated'].items() if v>3})" gpurun_out/ab_$2.json $2
}
run "$R/mantis_amd/libmantis_amd.so" base
for l in "$@"; do run "$R/$l" "$(basename $l .so)"; done
