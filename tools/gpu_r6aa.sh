#!/bin/bash
# GPU box: the lane DP's top stack slice kept in registers -- GPU tests, split
# phase ticks (previous / new), one-context stage times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06aa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
for k in 1 2; do for v in ts_prev ts_new; do
  echo "== $v"; MANTIS_AMD_LIB=$R/abvar/$v.so timeout -k 10 200 python -u tools/fc_ticks.py 1024 || exit 1
done; done | tee $O/fc_ticks.txt
bash tools/ab_kern.sh abvar/prev.so | tee $O/ab_kern.txt
