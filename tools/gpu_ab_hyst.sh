#!/bin/bash
# GPU box: parity of the changed stages, then A/B against alternative library
# builds (abvar/*.so) and k_frame_contours phase ticks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -k "canny or full_pipeline or throughput_mode or odd_capacity or contour or quads or border or detect" > gpurun_out/t_ab.txt 2>&1; rc=$?; tail -3 gpurun_out/t_ab.txt; [ $rc = 0 ] || exit 1
bash tools/ab_libs.sh abvar/*.so || exit 1
bash tools/ab_libs.sh abvar/*.so || exit 1
timeout -k 10 200 python -u tools/diag_contours.py 256 > gpurun_out/diag_contours.txt 2>&1; tail -6 gpurun_out/diag_contours.txt
