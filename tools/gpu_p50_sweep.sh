#!/bin/bash
# GPU box: single-rig latency (tools/p50_stages.py) under run-time switch sets,
# in-tree library. usage: tools/gpu_p50_sweep.sh "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/p50sw
i=0
for set in "" "$@" ""; do
  i=$((i+1))
  env $set timeout -k 10 120 python -u tools/p50_stages.py 48 > gpurun_out/p50sw/$i.json || exit 1
  python3 - gpurun_out/p50sw/$i.json "${set:-base}" <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
s = d["stages_median_ms"]
print(f"{sys.argv[2]:45s} p50 {d['p50_ms']:.3f} rpp_first {s['rpp_first']:.3f} rpp_cand {s['rpp_cand']:.3f} sum {d['stage_sum_ms']:.3f}", flush=True)
P
done
