#!/bin/bash
# GPU box, round 6 second call: GPU tests (Canny side-by-side strips, shift
# split fences), COLOR phase ticks, and isolated-stage A/B of the two changes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_b.txt 2>&1; rc=$?
tail -3 $O/gpu_tests_b.txt; [ $rc = 0 ] || exit 1
MANTIS_AMD_LIB=$R/abvar/ticks3.so timeout -k 10 120 python -u tools/score_ticks.py color 256 > $O/ticks_color.txt 2>&1 || exit 1
cat $O/ticks_color.txt
bash tools/ab_var.sh base=- catoff=-,MANTIS_CANNY_CAT=0 shsplit=-,MANTIS_SHIFT_SPLIT=1 \
  base2=- catoff2=-,MANTIS_CANNY_CAT=0 shsplit2=-,MANTIS_SHIFT_SPLIT=1 | tee $O/ab_b.txt
