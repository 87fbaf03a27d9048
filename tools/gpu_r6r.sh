#!/bin/bash
# GPU box: packed contour points (x | y << 16) with 8 / 4 / 6 points read
# ahead per lane in approxPolyDP -- GPU tests on the in-tree (8) build, the
# contour phase ticks, one-context stage times against the previous library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
for v in old pk4 pk6 new; do
  if [ $v = new ]; then lib=$R/mantis_amd/libmantis_amd.so; else lib=$R/abvar/$v.so; fi
  echo "== $v"; MANTIS_AMD_LIB=$lib timeout -k 10 200 python -u tools/fc_ticks.py 1024 || exit 1
done | tee $O/fc_ticks.txt
bash tools/ab_kern.sh abvar/old.so abvar/pk4.so abvar/pk6.so | tee $O/ab_kern.txt
