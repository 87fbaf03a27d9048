#!/bin/bash
# GPU box: the long borders' DP stack in LDS (in-tree) -- GPU tests, split
# phase ticks, one-context stage times against the previous build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
MANTIS_AMD_LIB=$R/abvar/ticksplit_stk.so timeout -k 10 200 python -u tools/fc_ticks.py 1024 | tee $O/fc_ticks.txt || exit 1
bash tools/ab_kern.sh abvar/prev.so | tee $O/ab_kern.txt
