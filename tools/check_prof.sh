#!/bin/bash
# GPU box: parity tests, then a rocprofv3 kernel-trace of one bench configuration.
# usage: tools/check_prof.sh TAG [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash "$R/tools/prof.sh" "$@"
