#!/bin/bash
# GPU box: GPU tests, then the bench legs (config 3 default with the CPU
# baseline, config 2, config 4, config 5), lines into gpurun_out/r03_bench_*.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; tail -3 gpurun_out/gpu_tests.log
fi
for leg in $LEGS; do
  case $leg in
    3) args="" ;;
    2) args="--config 2" ;;
    4) args="--config 4 --steps 5 --warmup 1 --latency-iters 3" ;;
    5) args="--config 5 --steps 20 --warmup 3" ;;
  esac
  timeout -k 10 400 python -u bench.py $args > gpurun_out/r03_bench_c$leg.log 2>&1 || { echo "bench $leg failed"; tail -20 gpurun_out/r03_bench_c$leg.log; exit 1; }
  grep '^{' gpurun_out/r03_bench_c$leg.log | tail -1 > gpurun_out/r03_bench_c$leg.json
  cut -c1-260 gpurun_out/r03_bench_c$leg.json
done
