#!/bin/bash
# GPU box: full GPU tests, smoke, default bench line, rocprofv3 kernel-trace
# summaries of the default bench (3 contexts) and of one context (isolated).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | tail -1 | cut -c1-400
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_default" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --ingest-steps 0 > "$R/gpurun_out/prof_default.log" 2>&1 || { echo "prof failed"; tail -20 "$R/gpurun_out/prof_default.log"; exit 1; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_c1" -o run -- python3 "$R/bench.py" --rigs 1024 --contexts 1 --steps 3 --warmup 1 --no-cpu --ingest-steps 0 > "$R/gpurun_out/prof_c1.log" 2>&1 || { echo "prof c1 failed"; tail -20 "$R/gpurun_out/prof_c1.log"; exit 1; }
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof_default gpurun_out/prof_default.md > /dev/null && python3 tools/prof_summary.py gpurun_out/prof_c1 gpurun_out/prof_c1.md > /dev/null && python3 tools/kern_avg.py gpurun_out/prof_c1/run_kernel_trace.csv > gpurun_out/kern_avg_c1.txt && python3 tools/kern_avg.py gpurun_out/prof_default/run_kernel_trace.csv 12 > gpurun_out/kern_avg_default.txt && head -12 gpurun_out/kern_avg_c1.txt
