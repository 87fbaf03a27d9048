#!/bin/bash
# GPU box: the fx:: Jacobi rotation in the product library -- GPU tests, the
# single-rig latency (hipGraph path) against the previous library, and a
# short default-bench A/B (rig poses/s and the isolated ObjPose stages).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
for k in 1 2; do
  MANTIS_AMD_LIB=$R/abvar/old.so timeout -k 10 120 python -u tools/p50_graph_ab.py 96 | sed 's/^/base /' || exit 1
  timeout -k 10 120 python -u tools/p50_graph_ab.py 96 | sed 's/^/fx   /' || exit 1
done | tee $O/p50_ab.txt
BSTEPS=8 bash tools/ab_var.sh base=abvar/old.so fx=- base2=abvar/old.so fx2=- | tee $O/ab.txt
