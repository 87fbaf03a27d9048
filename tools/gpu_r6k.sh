#!/bin/bash
# GPU box: border walks with a per-lane window of the tiled plane -- GPU tests,
# one-context stage times against the previous library, a short bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
bash tools/ab_kern.sh abvar/old.so abvar/win8.so | tee $O/ab_kern.txt || exit 1
BSTEPS=8 bash tools/ab_var.sh old=abvar/old.so new=- win8=abvar/win8.so old2=abvar/old.so new2=- win82=abvar/win8.so | tee $O/ab.txt
