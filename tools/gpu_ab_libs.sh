#!/bin/bash
# GPU box: A/B of the in-tree library against abvar/*.so builds (twice, alternating)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/ab_libs.sh abvar/*.so || exit 1
bash tools/ab_libs.sh abvar/*.so || exit 1
