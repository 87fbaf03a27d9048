#!/bin/bash
# GPU box, round 6 first call: the GPU tests (new switch fences included, the
# rig-latency hipGraphs with the runtime's packet capture off), smoke, the
# single-rig latency with / without graphs, the scoring phase ticks, and an
# A/B of scoring block shapes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_a.txt 2>&1; rc=$?
tail -3 $O/gpu_tests_a.txt; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_a.txt 2>&1 || { echo smoke failed; tail -5 $O/smoke_a.txt; exit 1; }
tail -1 $O/smoke_a.txt
for k in 1 2; do
  MANTIS_GRAPHS=0 timeout -k 10 120 python -u tools/p50_graph_ab.py 64 || exit 1
  timeout -k 10 120 python -u tools/p50_graph_ab.py 64 || exit 1
done | tee $O/p50_graph_ab.txt
MANTIS_AMD_LIB=$R/abvar/ticks1.so timeout -k 10 120 python -u tools/score_ticks.py 256 > $O/ticks_final.txt 2>&1 || exit 1
MANTIS_AMD_LIB=$R/abvar/ticks2.so timeout -k 10 120 python -u tools/score_ticks.py pf 256 > $O/ticks_pf.txt 2>&1 || exit 1
cat $O/ticks_final.txt $O/ticks_pf.txt
bash tools/ab_var.sh base=- glob=-,MANTIS_PF_MASK_GLOBAL=1 pf512g=abvar/pf512.so,MANTIS_PF_MASK_GLOBAL=1 \
  all512g=abvar/all512.so,MANTIS_PF_MASK_GLOBAL=1 base2=- pf512g2=abvar/pf512.so,MANTIS_PF_MASK_GLOBAL=1 \
  all512g2=abvar/all512.so,MANTIS_PF_MASK_GLOBAL=1 | tee $O/ab_a.txt
