#!/bin/bash
# GPU box: border-walk waves per frame (MK_TB_WAVES 2 / 8 builds against the
# in-tree 4), one-context stage times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp
bash tools/ab_kern.sh abvar/tbw2.so abvar/tbw8.so | tee $O/ab_kern.txt
