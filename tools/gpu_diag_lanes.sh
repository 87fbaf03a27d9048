set -o pipefail
mkdir -p gpurun_out/diag
for v in "MANTIS_OP_ROUNDS_SMALL=1" "MANTIS_OP_LANES_SMALL=1" "MANTIS_OP_LANES_SMALL=4 MANTIS_OP_ROUNDS_SMALL=1" "MANTIS_OP_LANES_SMALL=1 MANTIS_OP_ROUNDS_SMALL=1"; do
  env $v timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -q --timeout 120 --timeout-method thread -k "rig_gn_refines or paths_agree or rig_weighting" > gpurun_out/diag/t.txt 2>&1; rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/diag/t.txt)"
  [ $rc -le 1 ] || exit 1
done
bash tools/gpu_p50_sweep.sh "MANTIS_S1B_SPREAD_SMALL=64" "MANTIS_S1B_SPREAD_SMALL=8"
