#!/bin/bash
# GPU box: path halving in the band unions' LDS finds (halve build) -- GPU
# tests on it, one-context stage times against the in-tree library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06u; mkdir -p $O
export TMPDIR=/tmp
MANTIS_AMD_LIB=$R/abvar/halve.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_halve.txt 2>&1; rc=$?
tail -2 $O/gpu_tests_halve.txt; [ $rc = 0 ] || exit 1
bash tools/ab_kern.sh abvar/halve.so | tee $O/ab_kern.txt
