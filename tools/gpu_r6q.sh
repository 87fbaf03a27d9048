#!/bin/bash
# GPU box: single-rig latency against the HIP runtime's hardware queue count
# (bench.py sets GPU_MAX_HW_QUEUES = 4 x contexts = 24 for its six contexts).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06q; mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for q in 4 24; do
    echo -n "hwq $q: "; GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u tools/p50_ctx_probe.py 4096 5 64 || exit 1
  done
  for q in 8 16; do
    echo -n "hwq $q: "; GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u tools/p50_ctx_probe.py 4096 0 64 || exit 1
  done
done | tee $O/p50_hwq.txt
