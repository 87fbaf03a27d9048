#!/bin/bash
# GPU box: contour compaction with 2 points per lane (in-tree; 8 trips in
# flight: cpl2cu8) -- GPU tests, phase ticks, one-context stage times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
for v in prev cpl2cu8 new; do
  if [ $v = new ]; then lib=$R/mantis_amd/libmantis_amd.so; else lib=$R/abvar/$v.so; fi
  echo "== $v"; MANTIS_AMD_LIB=$lib timeout -k 10 200 python -u tools/fc_ticks.py 1024 || exit 1
done | tee $O/fc_ticks.txt
bash tools/ab_kern.sh abvar/prev.so abvar/cpl2cu8.so | tee $O/ab_kern.txt
