#!/bin/bash
# GPU box: border walks -- the next direction in registers (alu build), the
# walks on the row-major padded plane without k_tile_bits (rows build): GPU
# tests on both, one-context stage times, the checkpoint spacing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06m; mkdir -p $O
export TMPDIR=/tmp
for v in rows alu; do
  MANTIS_AMD_LIB=$R/abvar/$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_$v.txt 2>&1; rc=$?
  echo "$v: $(tail -1 $O/gpu_tests_$v.txt)"; [ $rc = 0 ] || exit 1
done
bash tools/ab_kern.sh abvar/rows.so abvar/alu.so MANTIS_SEG_M=32 MANTIS_SEG_M=96 | tee $O/ab_kern.txt
