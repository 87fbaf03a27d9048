#!/bin/bash
# PMC summary of every kernel of one bench configuration (GPU box), in
# rocprofv3 --pmc passes that each respect the per-block slot limits of
# MI355X_MICROARCH.md (one run per pass, counters filtered against
# `rocprofv3 -L`): instruction mix and wave states (SQ), MFMA (f64) activity,
# L2 hits / misses, HBM reads (FETCH_SIZE) and writes (WRITE_SIZE) in passes of
# their own. Per kernel: the launches with the largest grid (the batch
# launches), counters averaged per launch, FETCH_SIZE / WRITE_SIZE in bytes.
# Writes gpurun_out/pmc_$TAG.json with the library's lib_sha16 and its sources'
# src_sha16 (bench.py uses a summary only for the sources it was collected on).
# usage: tools/pmc_all.sh TAG [bench args...]   (default: --contexts 1 --rigs 256)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${1:-r04}; shift
BARGS=${*:-"--contexts 1 --rigs 256"}
export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
[ -s "$R/gpurun_out/counters_list.txt" ] || (cd /tmp && timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1) || true
have() { grep -qw "$1" "$R/gpurun_out/counters_list.txt"; }
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
  "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64"
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
  "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum"
  "TCP_TCC_READ_REQ_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i + 1))
  C=""
  for c in $P; do base=${c%_sum}; if have "$base" || have "$c"; then C="$C $c"; fi; done
  [ -n "$C" ] || continue
  echo "pass $i:$C"
  cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C -f csv -d "$OUT/p$i" -o run -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 --latency-iters 1 --ingest-steps 0 $BARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
cd "$R"
python3 - "$OUT" "$R/gpurun_out/pmc_$TAG.json" "$BARGS" <<'P'
import csv, glob, hashlib, json, os, re, sys, collections
out, dst, bargs = sys.argv[1], sys.argv[2], sys.argv[3]
def short(n):
    n = n.split("(")[0].replace("void ", "")
    n = n.split("::")[-1] if "::" in n.split("<")[0] else n
    return n.split("<")[0]
res = collections.defaultdict(dict)
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        by[short(r["Kernel_Name"])].append(r)
    for k, rs in by.items():
        g = max(int(r["Grid_Size"]) for r in rs)
        acc = collections.defaultdict(list)
        for r in rs:
            if int(r["Grid_Size"]) == g:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for c, v in acc.items():
            # one row per (dispatch, counter): the average over the batch launches
            val = sum(v) / len(v)
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                res[k][c + "_bytes"] = val * 1024.0  # kB -> bytes per launch
            else:
                res[k][c] = val
        res[k]["grid"] = g
for f in sorted(glob.glob(out + "/p1/**/*kernel_trace.csv", recursive=True)):
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        by[short(r["Kernel_Name"])].append((g, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    for k, v in by.items():
        gm = max(g for g, _ in v)
        sel = [t for g, t in v if g == gm]
        res[k]["duration_ms_profiled"] = sum(sel) / len(sel)
for k, d in res.items():
    wc = d.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in d:
                d[c + "_frac_of_wave_cycles"] = round(d[c] / wc, 4)
    if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
        d["tcc_hit_rate"] = round(d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"]), 4)
    if d.get("duration_ms_profiled") and "SQ_INSTS_VALU" in d:
        # wave64 VALU instruction = 2 cycles on a SIMD-32; 1024 SIMDs at 2.4 GHz
        d["valu_issue_frac"] = round(d["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9 * d["duration_ms_profiled"] * 1e-3), 4)
    if d.get("duration_ms_profiled") and "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
        d["mfma_busy_frac_of_gui_cycles"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, d["GRBM_GUI_ACTIVE"] * 256), 6)
fr = None
m = re.search(r"--rigs\s+(\d+)", bargs)
if m:
    fr = 4 * int(m.group(1))
root = os.environ.get("GRAFT_REPO_ROOT", ".")
sha = hashlib.sha256(open(os.path.join(root, "mantis_amd", "libmantis_amd.so"), "rb").read()).hexdigest()[:16]
sys.path.insert(0, root)
from bench import src_sha16
doc = {"lib_sha16": sha, "src_sha16": src_sha16(root), "bench_args": bargs, "frames_per_launch": fr,
       "note": "per kernel: batch launches (largest grid), counters averaged per launch; FETCH_SIZE_bytes as "
               "reported (gfx950: 1/2 of the bytes of 16-B coalesced reads, MI355X_MICROARCH.md), WRITE_SIZE_bytes "
               "as reported; valu_issue_frac = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x duration)",
       "kernels": res}
json.dump(doc, open(dst, "w"), indent=1, sort_keys=True)
for k, d in sorted(res.items(), key=lambda kv: -kv[1].get("duration_ms_profiled", 0))[:25]:
    print(k, json.dumps({c: (round(v, 4) if isinstance(v, float) else v) for c, v in sorted(d.items()) if c in (
        "duration_ms_profiled", "SQ_INSTS_VALU", "valu_issue_frac", "FETCH_SIZE_bytes", "WRITE_SIZE_bytes",
        "tcc_hit_rate", "SQ_WAIT_ANY_frac_of_wave_cycles", "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_VALU_MFMA_BUSY_CYCLES")}))
P
