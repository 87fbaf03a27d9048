#!/bin/bash
# GPU box: the round's compile-time alternatives still match the oracle --
# the GPU suite on builds with the long-border DP stack forced onto its
# global fallback (MK_WAVE_STK=2), the per-step walk loads (MK_WALK_WINDOW=0)
# and one point per lane in the contour compaction (MK_FC_CPL=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06z; mkdir -p $O
export TMPDIR=/tmp
for v in stk2 win0 cpl1; do
  MANTIS_AMD_LIB=$R/abvar/$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_$v.txt 2>&1; rc=$?
  echo "$v: $(tail -1 $O/gpu_tests_$v.txt)"; [ $rc = 0 ] || exit 1
done | tee $O/alternates.txt
