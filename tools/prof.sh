#!/bin/bash
# rocprofv3 kernel trace + stats of one bench configuration (GPU box)
# usage: tools/prof.sh TAG [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv rocpd -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { echo "prof failed"; tail -30 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
grep '^{' "$R/gpurun_out/prof_$TAG.log" | tail -1
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_$TAG.md" | head -30
