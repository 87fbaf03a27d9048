#!/bin/bash
# GPU box: the default bench three more times on the final sources (no CPU
# leg), for the run-to-run spread of the committed line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06rep; mkdir -p $O
export TMPDIR=/tmp
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu > $O/b$k.log 2>&1 || { tail -3 $O/b$k.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('run', sys.argv[2], 'rig poses/s', d['value'], 'ms/step', d['ms_per_step'], 'published/s', d['published_rig_poses_per_s'], 'p50', d['p50_latency_ms'], 'src', d['src_sha16'])" $O/b$k.log $k
done | tee $O/repeats.txt
