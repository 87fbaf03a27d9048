#!/bin/bash
# HBM traffic of the Canny front-end kernel (GPU box): FETCH_SIZE and WRITE_SIZE
# in separate passes (MI355X_MICROARCH.md: they do not fit one pass), 256
# frames per launch; writes gpurun_out/pmc_traffic.json (bytes per frame).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -f csv -d "$R/gpurun_out/pmc_$C" -o run -- python3 "$R/bench.py" --no-cpu --rigs 64 --contexts 1 --steps 2 --warmup 1 --latency-iters 1 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_$C.log"; exit 1; }
done
python3 - "$R/gpurun_out" <<'P'
import csv, glob, json, sys
out = {"stage": "canny_nms", "kernel": "k_canny_uf"}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{sys.argv[1]}/pmc_{c}/**/*counter_collection.csv", recursive=True)[0]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if r["Kernel_Name"].startswith("mk::k_canny_uf") and int(r["Grid_Size"]) == 10 * 45 * 256 * 256]
    out[c + "_kB_per_launch"] = sum(vals) / len(vals)
    out["launches_" + c] = len(vals)
# FETCH_SIZE/WRITE_SIZE are in kB; FETCH_SIZE counts half of wide coalesced reads on gfx950
out["fetch_raw_bytes_per_frame"] = out["FETCH_SIZE_kB_per_launch"] * 1024 / 256
fetch = out["FETCH_SIZE_kB_per_launch"] * 1024 * 2
write = out["WRITE_SIZE_kB_per_launch"] * 1024
out["hbm_bytes_per_frame"] = (fetch + write) / 256
out["note"] = "FETCH_SIZE doubled (gfx950 correction for wide coalesced reads; 12-byte-per-lane loads are uncalibrated), WRITE_SIZE as reported; per frame of 1280x720"
json.dump(out, open(f"{sys.argv[1]}/pmc_traffic.json", "w"), indent=1)
print(json.dumps(out))
P
