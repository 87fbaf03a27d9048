#!/bin/bash
# GPU box: the default (6-context) bench, short, for the in-tree library and
# variants, alternating twice: an argument VAR=value sets that environment
# variable, anything else is an alternative library (MANTIS_AMD_LIB).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {  # tag [VAR=value | lib.so]
  local tag=$1 v=$2
  local envs=() lib="$R/mantis_amd/libmantis_amd.so"
  case "$v" in *=*) envs=("$v") ;; "") ;; *) lib="$R/$v" ;; esac
  env "${envs[@]}" MANTIS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --latency-iters 5 --no-cpu --ingest-steps 0 > gpurun_out/abf_$tag.json 2> gpurun_out/abf_$tag.err || { tail -5 gpurun_out/abf_$tag.err; return 1; }
  python3 - gpurun_out/abf_$tag.json $tag <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], d["value"], "p50", d["p50_latency_ms"], "cpu/step", d.get("host_cpu_s_per_step"),
      {k: round(v, 2) for k, v in r["stages_ms_isolated"].items() if v > 1.0}, flush=True)
P
}
for rep in 1 2; do
  run base "" || exit 1
  for v in "$@"; do run "$(echo $v | tr -c 'A-Za-z0-9_\n' '_')" "$v" || exit 1; done
done
