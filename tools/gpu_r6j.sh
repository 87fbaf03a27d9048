#!/bin/bash
# GPU box: the fx:: Jacobi rotation with a per-rotation library fallback --
# the single-lane probe (fx / library builds, bit for bit), GPU tests, the
# single-rig latency against the previous library and a short bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r06j; mkdir -p $O
export TMPDIR=/tmp
OBJPOSE_LAT_OUT=$O/lat_lib.bin timeout -k 10 120 ./tools/objpose_lat_lib > $O/lat_lib.txt || { tail -3 $O/lat_lib.txt; exit 1; }
OBJPOSE_LAT_OUT=$O/lat_fx.bin timeout -k 10 120 ./tools/objpose_lat_fx > $O/lat_fx.txt || { tail -3 $O/lat_fx.txt; exit 1; }
tail -1 $O/lat_lib.txt; tail -1 $O/lat_fx.txt
cmp $O/lat_lib.bin $O/lat_fx.bin > /dev/null && echo "device results identical incl. timings?" || python3 - $O/lat_lib.bin $O/lat_fx.bin <<'PY'
import sys
a = open(sys.argv[1], 'rb').read(); b = open(sys.argv[2], 'rb').read()
rec = 136
diff = [i for i in range(len(a) // rec) if a[i*rec:i*rec+112] != b[i*rec:i*rec+112] or a[i*rec+128:(i+1)*rec] != b[i*rec+128:(i+1)*rec]]
print('device lib vs fx: %d problems, %d differ %s' % (len(a) // rec, len(diff), diff))
sys.exit(1 if diff else 0)
PY
[ $? = 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt; [ $rc = 0 ] || exit 1
for k in 1 2; do
  MANTIS_AMD_LIB=$R/abvar/old.so timeout -k 10 120 python -u tools/p50_graph_ab.py 96 | sed 's/^/base /' || exit 1
  timeout -k 10 120 python -u tools/p50_graph_ab.py 96 | sed 's/^/fx   /' || exit 1
done | tee $O/p50_ab.txt
BSTEPS=8 bash tools/ab_var.sh base=abvar/old.so fx=- base2=abvar/old.so fx2=- | tee $O/ab.txt
