#!/bin/bash
# bench sweep over batch size / contexts (GPU box); one line per config into gpurun_out/sweep.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
: > gpurun_out/sweep.log
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/sweep.log
  timeout -k 10 300 python bench.py --no-cpu --latency-iters 3 $cfg >> gpurun_out/sweep.log 2>&1 || { echo "failed: $cfg"; tail -20 gpurun_out/sweep.log; exit 1; }
done
python - <<'P'
import json
for l in open('gpurun_out/sweep.log'):
    if l.startswith('=='): print(l.strip(), end=' ')
    elif l.startswith('{'):
        d=json.loads(l); r=d.get('roofline') or {}; print(d['value'], d['ms_per_step'], d['p50_latency_ms'], r.get('kernel'), r.get('achieved'), r.get('unit'), json.dumps(r.get('stages_ms')))
P
