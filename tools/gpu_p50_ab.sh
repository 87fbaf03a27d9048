#!/bin/bash
# GPU box: single-rig latency A/B of run-time switches: per-stage medians
# (tools/p50_stages.py) and the bench's p50 (tools/ab_kern.sh), in-tree library.
# usage: tools/gpu_p50_ab.sh VAR=value ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/p50ab
for rep in 1 2; do
  timeout -k 10 120 python -u tools/p50_stages.py 48 > gpurun_out/p50ab/base_$rep.json || exit 1
  echo "base $(cat gpurun_out/p50ab/base_$rep.json)"
  for kv in "$@"; do
    env "$kv" timeout -k 10 120 python -u tools/p50_stages.py 48 > gpurun_out/p50ab/alt_$rep.json || exit 1
    echo "$kv $(cat gpurun_out/p50ab/alt_$rep.json)"
  done
done
timeout -k 10 400 bash tools/ab_kern.sh "$@"
