#!/bin/bash
# GPU-box check: parity tests, smoke, bench line, rocprofv3 kernel-trace summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv rocpd -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/prof.log" 2>&1 || { echo "prof failed"; tail -30 "$R/gpurun_out/prof.log"; exit 1; }
  grep '^{' "$R/gpurun_out/prof.log" | tail -1
  python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof" "$R/gpurun_out/prof.md"
fi
