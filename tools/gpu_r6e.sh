#!/bin/bash
# GPU box: scoring tests after moving the 81 shifts into k_score_pf, then one-context A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_switches.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "scor or full_pipeline or mixed or switches or throughput or latency or two_rig or config or mask" > $O/gpu_tests_e.txt 2>&1; rc=$?
tail -3 $O/gpu_tests_e.txt; [ $rc = 0 ] || exit 1
bash tools/ab_kern.sh abvar/prev.so
