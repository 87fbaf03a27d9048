#!/bin/bash
# GPU box: where k_frame_contours' DP time goes (long borders on waves vs
# short ones on lanes: tick-split build) and the border length statistics;
# GPU tests on the in-tree build (compaction at 8 trips in flight).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
MANTIS_AMD_LIB=$R/abvar/ticksplit.so timeout -k 10 200 python -u tools/fc_ticks.py 1024 | tee $O/fc_ticks_split.txt || exit 1
timeout -k 10 200 python -u tools/fc_stats.py 64 | tee $O/fc_stats.txt
