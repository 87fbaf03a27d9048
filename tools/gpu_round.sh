#!/bin/bash
# GPU-box check: parity tests, bench line, rocprofv3 kernel-trace summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv rocpd -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/prof.log" 2>&1 || { echo "prof failed"; tail -30 "$R/gpurun_out/prof.log"; exit 1; }
  ls -R "$R/gpurun_out/prof"
fi
