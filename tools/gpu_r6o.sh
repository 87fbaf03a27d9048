#!/bin/bash
# GPU box: single-rig latency against context 0's size and idle contexts
# beside it (tools/p50_ctx_probe.py), twice each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for cfg in "4096 0" "4096 5" "4 5"; do
    timeout -k 10 240 python -u tools/p50_ctx_probe.py $cfg 64 || exit 1
  done
done | tee $O/p50_ctx.txt
