#!/bin/bash
# GPU box: shard fixture, GPU tests, screen validation, library A/B, score PMC
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
if [ -n "$FIXTURE" ]; then
  timeout -k 10 300 python -u tests/golden/make_shard_fixture.py gpurun_out/shard_batch.npz > gpurun_out/shard_fixture.log 2>&1 || { echo "fixture failed"; tail -20 gpurun_out/shard_fixture.log; exit 1; }
  tail -1 gpurun_out/shard_fixture.log
fi
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; tail -3 gpurun_out/gpu_tests.log
[ -s gpurun_out/map.txt ] || python3 -c "from mantis_amd import synth; import numpy as np; w,r,g=synth.load_map(); np.savetxt('gpurun_out/map.txt', np.vstack([w,r,g]))"
[ -n "$NOSCREEN" ] || timeout -k 10 200 ./tools/check_screen 134217728 gpurun_out/map.txt | tail -4 || exit 1
bash tools/ab_libs.sh "$@"
[ -n "$NOPMC" ] || bash tools/pmc_score.sh ${PMCTAG:-scr2} k_score > gpurun_out/pmc_scr2.txt 2>&1; tail -1 gpurun_out/pmc_scr2.txt | cut -c1-200
