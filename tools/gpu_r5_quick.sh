mkdir -p gpurun_out/r05 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_hysteresis.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/r05/t3.log 2>&1; rc=$?; tail -3 gpurun_out/r05/t3.log; [ $rc = 0 ] || exit 1
(cd /tmp && timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r05/calib_f -o run -- $GRAFT_REPO_ROOT/tools/pmc_calib > $GRAFT_REPO_ROOT/gpurun_out/r05/calib_f.log 2>&1) || echo calib f failed
(cd /tmp && timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r05/calib_w -o run -- $GRAFT_REPO_ROOT/tools/pmc_calib > $GRAFT_REPO_ROOT/gpurun_out/r05/calib_w.log 2>&1) || echo calib w failed
timeout -k 10 300 bash tools/ab_kern.sh 2>&1 | tail -2
timeout -k 10 500 python -u bench.py --no-cpu --ingest-steps 0 > gpurun_out/r05/bench_quick.log 2>&1 || exit 1
grep "^{" gpurun_out/r05/bench_quick.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_ms']); r=d['roofline']; print(r['stages_ms']); print(r.get('stages_ms_isolated'))"
