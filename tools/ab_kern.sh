#!/bin/bash
# GPU box: one-context stage / kernel times (1024 rigs = 4096 frames per launch)
# of the in-tree library and of alternative builds, twice each, alternating.
# usage: tools/ab_kern.sh [lib.so ...]   (env BARGS: extra bench args)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {
  MANTIS_AMD_LIB=$1 timeout -k 10 200 python -u bench.py --contexts 1 --rigs 1024 --steps 3 --warmup 1 --latency-iters 3 --no-cpu --ingest-steps 0 $BARGS > gpurun_out/abk_$2.json 2> gpurun_out/abk_$2.err || { tail -5 gpurun_out/abk_$2.err; exit 1; }
  python3 - gpurun_out/abk_$2.json $2 <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
st = {k: round(v, 2) for k, v in r["stages_ms"].items() if v > 0.5}
print(sys.argv[2], "p50", d["p50_latency_ms"], "kern", r.get("kernels_ms"), st, flush=True)
P
}
# an argument VAR=value runs the in-tree library with that environment variable
for rep in 1 2; do
  run "$R/mantis_amd/libmantis_amd.so" base || exit 1
  for l in "$@"; do
    case "$l" in
      *=*) env "$l" bash -c "true" && export "$l" && run "$R/mantis_amd/libmantis_amd.so" "${l//[^A-Za-z0-9_]/_}"; rc=$?; unset "${l%%=*}"; [ $rc = 0 ] || exit 1 ;;
      *) run "$R/$l" "$(basename $l .so)" || exit 1 ;;
    esac
  done
done
