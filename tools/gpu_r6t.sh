#!/bin/bash
# GPU box: k_frame_contours waves per SIMD (4: 128 VGPRs) and approxPolyDP
# read-ahead (16 packed points), one-context stage times and phase ticks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06t; mkdir -p $O
export TMPDIR=/tmp
for v in wpe4k8 wpe4k16 wpe5k16 new; do
  if [ $v = new ]; then lib=$R/mantis_amd/libmantis_amd.so; else lib=$R/abvar/$v.so; fi
  echo "== $v"; MANTIS_AMD_LIB=$lib timeout -k 10 200 python -u tools/fc_ticks.py 1024 || exit 1
done | tee $O/fc_ticks.txt
bash tools/ab_kern.sh abvar/wpe4k8.so abvar/wpe4k16.so abvar/wpe5k16.so | tee $O/ab_kern.txt
