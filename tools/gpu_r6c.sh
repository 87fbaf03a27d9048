#!/bin/bash
# GPU box: k_score_final phase ticks (shift tasks, COLOR) of the current sources
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06; mkdir -p $O
MANTIS_AMD_LIB=$R/abvar/ticks3.so timeout -k 10 120 python -u tools/score_ticks.py color 256 > $O/ticks_color2.txt 2>&1 || exit 1
MANTIS_AMD_LIB=$R/abvar/ticks1.so timeout -k 10 120 python -u tools/score_ticks.py 256 > $O/ticks_final2.txt 2>&1 || exit 1
cat $O/ticks_color2.txt $O/ticks_final2.txt
