#!/bin/bash
# GPU box: contexts per GPU at a fixed 6144 rigs per step (fused rig GN default)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
export BSTEPS=12
bash tools/ab_var.sh c6=- || exit 1
BARGS="--contexts 8 --rigs 6144" bash tools/ab_var.sh c8=- || exit 1
BARGS="--contexts 4 --rigs 6144" bash tools/ab_var.sh c4=- || exit 1
bash tools/ab_var.sh c6b=- || exit 1
BARGS="--contexts 8 --rigs 6144" bash tools/ab_var.sh c8b=- || exit 1
