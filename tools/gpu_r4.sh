#!/bin/bash
# GPU box, round 4: parity tests, the default bench line, and optionally a
# one-context rocprofv3 kernel trace (PROF=1) / the all-kernel PMC passes (PMC=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/${TAG:-r04}; mkdir -p $O
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
  tail -3 $O/gpu_tests.txt; [ $rc = 0 ] || { grep -E "FAIL|Error|error" $O/gpu_tests.txt | head -20; exit 1; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py --no-cpu --ingest-steps 0 ${BARGS} > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | tail -1 > $O/bench.json
  python3 - $O/bench.json <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "p50", d["p50_latency_ms"], "host_cpu_s/step", d.get("host_cpu_s_per_step"))
print("dom", r["kernel"], r["avg_launch_ms"], r.get("kernels_ms"), "frac", r["frac"])
print("iso", r.get("isolated"))
print("stages_iso", r.get("stages_ms_isolated"))
P
fi
if [ "${PROF:-0}" = 1 ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/$O/prof_c1" -o run -- python3 "$R/bench.py" --no-cpu --contexts 1 --steps 3 --warmup 1 --latency-iters 3 --ingest-steps 0 > "$R/$O/prof_c1.log" 2>&1) || { echo prof c1 failed; tail -5 $O/prof_c1.log; exit 1; }
  python3 tools/kern_avg.py $O/prof_c1/run_kernel_trace.csv 40 $O/batch_launch_avg_c1.json > $O/batch_launch_avg_c1.txt
  head -30 $O/batch_launch_avg_c1.txt
fi
if [ "${PMC:-0}" = 1 ]; then
  bash tools/pmc_all.sh ${TAG:-r04} > $O/pmc.log 2>&1 || { echo pmc failed; tail -20 $O/pmc.log; exit 1; }
  tail -25 $O/pmc.log
fi
