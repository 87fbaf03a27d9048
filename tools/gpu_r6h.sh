#!/bin/bash
# GPU box: ObjPose footprint under the 6-context load (2 waves per SIMD; fewer blocks)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
export BSTEPS=12
bash tools/ab_var.sh base=- opw2=abvar/opw2.so b32=-,MANTIS_RPP_BLOCKS=32 b48=-,MANTIS_RPP_BLOCKS=48 \
  base2=- opw2b=abvar/opw2.so b32b=-,MANTIS_RPP_BLOCKS=32 b48b=-,MANTIS_RPP_BLOCKS=48
