#!/bin/bash
# GPU box, round-6 evidence. PART=a: GPU tests, smoke, default bench line (with
# the CPU baseline), one-context kernel trace; PART=b: rocprofv3 kernel trace +
# stats of the default command, batch-launch averages, and the config 2 / 5 / 4
# legs; PART=d: every kernel's PMC summary (tools/pmc_all.sh, digest-tagged:
# bench.py reads traffic / VALU issue from it for these sources only); PART=da:
# d, then a with that summary in place.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06; mkdir -p $O
export TMPDIR=/tmp
if [ "$PART" = "d" ] || [ "$PART" = "da" ]; then
  bash tools/pmc_all.sh r06 > $O/pmc.log 2>&1 || { echo pmc failed; tail -20 $O/pmc.log; exit 1; }
  cp gpurun_out/pmc_r06.json $O/pmc_r06.json
  tail -3 $O/pmc.log
  # the bench line below reads this summary (same sources) for traffic / VALU issue
  [ "$PART" = "da" ] && cp gpurun_out/pmc_r06.json profiles/r06_pmc.json
fi
if [ "$PART" = "a" ] || [ "$PART" = "da" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; tail -2 $O/gpu_tests.txt
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && tail -1 $O/smoke.txt || { echo smoke failed; tail -5 $O/smoke.txt; exit 1; }
  timeout -k 10 700 python -u bench.py > $O/bench_default.log 2>&1 || { echo bench failed; tail -5 $O/bench_default.log; exit 1; }
  grep '^{' $O/bench_default.log | tail -1 > $O/bench_default.json; cut -c1-200 $O/bench_default.json
fi
if [ "$PART" = "b" ]; then
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$R/$O/prof_default" -o run -- python3 "$R/bench.py" --no-cpu --steps 3 --warmup 1 --latency-iters 3 --ingest-steps 0 > "$R/$O/prof_default.log" 2>&1) || { echo prof failed; tail -5 $O/prof_default.log; exit 1; }
  python3 tools/prof_summary.py $O/prof_default $O/rocprof_stats_default.md > /dev/null
  python3 tools/kern_avg.py $O/prof_default/run_kernel_trace.csv 40 $O/batch_launch_avg_default.json > $O/batch_launch_avg_default.txt
  python3 tools/trace_overlap.py $O/prof_default 18 > $O/trace_overlap_default.txt || true
  python3 tools/dur_sources.py $O/prof_default $O/prof_default.log > $O/duration_sources.txt || true
  head -12 $O/batch_launch_avg_default.txt
  for leg in 2 5 4; do
    case $leg in
      2) args="--config 2" ;;
      4) args="--config 4 --steps 5 --warmup 1 --latency-iters 3" ;;
      5) args="--config 5 --steps 20 --warmup 3" ;;
    esac
    timeout -k 10 400 python -u bench.py $args > $O/bench_c$leg.log 2>&1 || { echo "bench $leg failed"; tail -5 $O/bench_c$leg.log; exit 1; }
    grep '^{' $O/bench_c$leg.log | tail -1 > $O/bench_c$leg.json; cut -c1-160 $O/bench_c$leg.json
  done
fi
if [ "$PART" = "a" ] || [ "$PART" = "da" ] || [ "$PART" = "c" ]; then
  # one context: the kernels' own durations without the other contexts' blocks
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/$O/prof_c1" -o run -- python3 "$R/bench.py" --no-cpu --contexts 1 --steps 3 --warmup 1 --latency-iters 3 --ingest-steps 0 > "$R/$O/prof_c1.log" 2>&1) || { echo prof c1 failed; tail -5 $O/prof_c1.log; exit 1; }
  python3 tools/prof_summary.py $O/prof_c1 $O/rocprof_stats_c1.md > /dev/null
  python3 tools/kern_avg.py $O/prof_c1/run_kernel_trace.csv 40 $O/batch_launch_avg_c1.json > $O/batch_launch_avg_c1.txt
  head -30 $O/batch_launch_avg_c1.txt
fi
