#!/bin/bash
# GPU box: short default bench at several context counts (and rig counts).
# usage: tools/sweep_ctx.sh "CTX:RIGS" ...   e.g. 2:3072 3:3072 4:3072
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for cr in "$@"; do
  c=${cr%%:*}; r=${cr##*:}
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 2 --latency-iters 1 --no-cpu --ingest-steps 0 --contexts $c --rigs $r > gpurun_out/ctx_$c_$r.json 2> gpurun_out/ctx_${c}_$r.err || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step'],{k:round(v,1) for k,v in d['roofline']['stages_ms'].items() if v>5})" gpurun_out/ctx_$c_$r.json "ctx=$c rigs=$r"
done
