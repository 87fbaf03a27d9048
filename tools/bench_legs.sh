#!/bin/bash
# GPU box: default bench line (config 3 + host ingest + CPU baseline), then the config 4 / 5 legs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench3.log 2>&1 || { echo "bench3 failed"; tail -30 gpurun_out/bench3.log; exit 1; }
grep '^{' gpurun_out/bench3.log | tail -1
timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 1 > gpurun_out/bench4.log 2>&1 || { echo "bench4 failed"; tail -30 gpurun_out/bench4.log; exit 1; }
grep '^{' gpurun_out/bench4.log | tail -1
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/bench5.log 2>&1 || { echo "bench5 failed"; tail -30 gpurun_out/bench5.log; exit 1; }
grep '^{' gpurun_out/bench5.log | tail -1
