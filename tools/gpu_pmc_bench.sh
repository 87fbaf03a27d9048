#!/bin/bash
# Per-kernel PMC of the default bench command (measurement; GPU box):
# pass 1 VALU / SALU / LDS / VMEM instruction counts and wave cycles, pass 2
# HBM bytes. Writes gpurun_out/pmc_bench{1,2}/ (CSV counter collections).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/pmc_bench1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 --latency-iters 2 --ingest-steps 0 \
  > "$R/gpurun_out/pmc_bench1.log" 2>&1 || { echo pass1 failed; tail -5 "$R/gpurun_out/pmc_bench1.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE \
  -d "$R/gpurun_out/pmc_bench2" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 --latency-iters 2 --ingest-steps 0 \
  > "$R/gpurun_out/pmc_bench2.log" 2>&1 || { echo pass2 failed; tail -5 "$R/gpurun_out/pmc_bench2.log"; exit 1; }
echo pmc done
