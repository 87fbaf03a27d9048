#!/bin/bash
# HBM traffic of the Canny front-end and hysteresis kernels (GPU box):
# FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md: they do
# not fit one pass), 256 frames per launch (707 MB of BGR input: past the
# 256 MiB Infinity Cache); writes gpurun_out/pmc_traffic.json (bytes per frame).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $C -f csv -d "$R/gpurun_out/pmc_$C" -o run -- python3 "$R/bench.py" --no-cpu --rigs 64 --contexts 1 --steps 2 --warmup 1 --latency-iters 1 --ingest-steps 0 > "$R/gpurun_out/pmc_$C.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_$C.log"; exit 1; }
done
python3 - "$R/gpurun_out" <<'P'
import csv, glob, json, sys
FR = 256
kern = {"canny_nms": ["k_canny_strip", "k_canny"], "hysteresis": ["k_hyst_band", "k_hyst_seam", "k_hyst_mark", "k_hyst_fix"]}
out = {"stage": "canny_nms", "kernel": "k_canny_strip", "frames_per_launch": FR}
per = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{sys.argv[1]}/pmc_{c}/**/*counter_collection.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    for stage, names in kern.items():
        tot = 0.0
        for k in names:
            sel = [r for r in rows if r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0] == "mk::" + k]
            if not sel:
                continue
            g = max(int(r["Grid_Size"]) for r in sel)
            vals = [float(r["Counter_Value"]) for r in sel if int(r["Grid_Size"]) == g]
            v = sum(vals) / len(vals) * 1024 / FR  # kB per launch -> bytes per frame
            per[f"{k}_{c}_bytes_per_frame"] = round(v)
            tot += v
        per[f"{stage}_{c}_bytes_per_frame"] = round(tot)
out.update(per)
# calibration (tools/pmc_calib.hip, profiles/r02_pmc_calib.txt): FETCH_SIZE reports 1/2 of the bytes of
# 12- and 16-byte-per-lane reads. The 2x WRITE_SIZE of 16-byte tile-row stores measured there came from
# neighbouring tiles' partial sectors written back by different XCDs' L2s; with the XCD-aware tile order
# the neighbours share an L2 and WRITE_SIZE equals the bit-plane bytes (2 x W H / 8), so it is taken as is.
out["canny_nms_hbm_bytes_per_frame"] = 2 * per["canny_nms_FETCH_SIZE_bytes_per_frame"] + per["canny_nms_WRITE_SIZE_bytes_per_frame"]
out["hysteresis_hbm_bytes_per_frame"] = 2 * per["hysteresis_FETCH_SIZE_bytes_per_frame"] + per["hysteresis_WRITE_SIZE_bytes_per_frame"]
out["hbm_bytes_per_frame"] = out["canny_nms_hbm_bytes_per_frame"]
out["note"] = ("per 1280x720 frame; k_canny_strip: FETCH_SIZE x 2 (calibrated on 12-byte reads, tools/pmc_calib.hip; the strip kernel reads 12 bytes per column group) "
               "+ WRITE_SIZE (= the 2 x W H / 8 bit-plane bytes); hysteresis: FETCH_SIZE x 2 + WRITE_SIZE "
               "(its access widths uncalibrated); algorithmic k_canny bytes: 3 W H + W H / 4 = 2,995,200")
json.dump(out, open(f"{sys.argv[1]}/pmc_traffic.json", "w"), indent=1)
print(json.dumps(out))
P
