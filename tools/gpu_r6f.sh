#!/bin/bash
# GPU box: RPP tests after the per-round ObjPose counters, then 6-context A/B
# against the previous build and a contexts-per-GPU sweep at 6144 rigs per step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_switches.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "rpp or objpose or full_pipeline or switches or two_rig or config4" > $O/gpu_tests_f.txt 2>&1; rc=$?
tail -2 $O/gpu_tests_f.txt; [ $rc = 0 ] || exit 1
export BSTEPS=12
bash tools/ab_var.sh c6=- prev=abvar/prev.so c6b=- prevb=abvar/prev.so || exit 1
BARGS="--contexts 8 --rigs 6144" bash tools/ab_var.sh c8=- || exit 1
BARGS="--contexts 4 --rigs 6144" bash tools/ab_var.sh c4=- || exit 1
