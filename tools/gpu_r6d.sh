#!/bin/bash
# GPU box: border-walk tests on the round-6 tile layout, then one-context stage times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_switches.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "contour or border or segmented or morphology or many_borders or throughput or full_pipeline or mixed" > $O/gpu_tests_d.txt 2>&1; rc=$?
tail -3 $O/gpu_tests_d.txt; [ $rc = 0 ] || exit 1
bash tools/ab_kern.sh
