#!/bin/bash
# GPU box: walk-window variants (4 words in-tree, 8 words, 8 words placed
# ahead in x and y): the border-walk and pipeline GPU tests on the 8h build,
# one-context stage times, a short bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06l; mkdir -p $O
export TMPDIR=/tmp
MANTIS_AMD_LIB=$R/abvar/win8h.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_8h.txt 2>&1; rc=$?
tail -3 $O/gpu_tests_8h.txt; [ $rc = 0 ] || exit 1
bash tools/ab_kern.sh abvar/win8.so abvar/win8h.so | tee $O/ab_kern.txt || exit 1
BSTEPS=8 bash tools/ab_var.sh old=abvar/old.so new=- win8h=abvar/win8h.so old2=abvar/old.so new2=- win8h2=abvar/win8h.so | tee $O/ab.txt
