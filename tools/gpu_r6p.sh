#!/bin/bash
# GPU box: bench.py's config-3 p50 after a short and after the default
# throughput phase (is the rig latency lower on a GPU that has not just run
# six contexts flat out?).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06p; mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for st in "1 0" "10 2"; do
    set -- $st
    timeout -k 10 300 python -u bench.py --no-cpu --ingest-steps 0 --steps $1 --warmup $2 > $O/b_$1_$k.log 2>&1 || { tail -3 $O/b_$1_$k.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('steps', sys.argv[2], 'value', d['value'], 'p50', d['p50_latency_ms'], 'rig0', d['p50_latency_rig0_ms'])" $O/b_$1_$k.log $1
  done
done | tee $O/p50_after_load.txt
