#!/bin/bash
# GPU box: border-walk chunks stored packed (x | y << 16, half the bytes) --
# GPU tests, one-context stage times against the previous build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
bash tools/ab_kern.sh abvar/prev.so | tee $O/ab_kern.txt
