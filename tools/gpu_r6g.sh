#!/bin/bash
# GPU box: morphology tests with the mask chain split over waves, one-context A/B of the split
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_switches.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "morph or detector or throughput_path or contour or full_pipeline" > $O/gpu_tests_g.txt 2>&1; rc=$?
tail -2 $O/gpu_tests_g.txt; [ $rc = 0 ] || exit 1
bash tools/ab_kern.sh MANTIS_MORPH_MASK_SEGS=1 MANTIS_MORPH_MASK_SEGS=3 MANTIS_MORPH_MASK_SEGS=4
