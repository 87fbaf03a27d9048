#!/bin/bash
# GPU box: short default-bench A/B of library builds and run-time settings.
# usage: tools/ab_var.sh name=lib.so[,ENV=VAL,...] ...  (lib "-" = the in-tree library)
# Prints per variant: rig poses/s and the isolated stages above 1 ms.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}
  IFS=, read -r lib envs <<< "$rest"
  [ "$lib" = "-" ] && lib=mantis_amd/libmantis_amd.so
  envcmd=(env MANTIS_AMD_LIB="$R/$lib")
  if [ -n "$envs" ]; then IFS=, read -ra kv <<< "$envs"; envcmd+=("${kv[@]}"); fi
  timeout -k 10 180 "${envcmd[@]}" python -u bench.py --steps ${BSTEPS:-5} --warmup 2 --latency-iters 1 --no-cpu --ingest-steps 0 $BARGS \
    > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || { echo "$name failed"; tail -3 gpurun_out/ab/$name.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], d['value'], {k:round(v,2) for k,v in r['stages_ms_isolated'].items() if v>1}, 'kern', r.get('kernels_ms'))
" gpurun_out/ab/$name.json "$name"
done
