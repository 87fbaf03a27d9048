#!/bin/bash
# PMC evidence for the scoring kernels (GPU box): several rocprofv3 --pmc
# passes (each within the per-block slot limits of MI355X_MICROARCH.md, one
# run each, counters filtered against `rocprofv3 -L`) over a short
# single-context bench run (1024 frames per launch), summarised per kernel
# (batch launches = the largest grid) into gpurun_out/pmc_score_$TAG.json.
# usage: tools/pmc_score.sh TAG [kernel regex] [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${1:-base}; KRE=${2:-k_score}; shift 2 2>/dev/null
BARGS=${*:-"--rigs 256"}
export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_score_$TAG"
mkdir -p "$OUT"
[ -s "$R/gpurun_out/counters_list.txt" ] || (cd /tmp && timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1) || true
have() { grep -qw "$1" "$R/gpurun_out/counters_list.txt"; }
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
  "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64"
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
  "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i + 1))
  C=""
  for c in $P; do base=${c%_sum}; if have "$base" || have "$c"; then C="$C $c"; fi; done
  [ -n "$C" ] || continue
  echo "pass $i:$C"
  cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C -f csv -d "$OUT/p$i" -o run -- python3 "$R/bench.py" --no-cpu --contexts 1 --steps 2 --warmup 1 --latency-iters 1 --ingest-steps 0 $BARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" "$KRE" "$R/gpurun_out/pmc_score_$TAG.json" <<'P'
import csv, glob, json, re, sys, collections
out, kre, dst = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3]
res = collections.defaultdict(dict)
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if kre.search(r["Kernel_Name"])]
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(r)
    for k, rs in by.items():
        g = max(int(r["Grid_Size"]) for r in rs)
        acc = collections.defaultdict(list)
        for r in rs:
            if int(r["Grid_Size"]) == g:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for c, v in acc.items():
            res[k][c] = sum(v) / len(v)
        res[k]["grid"] = g
for f in sorted(glob.glob(out + "/p1/**/*kernel_trace.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if kre.search(r["Kernel_Name"])]
    by = collections.defaultdict(list)
    for r in rows:
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        by[r["Kernel_Name"].split("(")[0].replace("void ", "")].append((g, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
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
    if "GRBM_GUI_ACTIVE" in d and d.get("duration_ms_profiled"):
        d["eff_clock_GHz"] = round(d["GRBM_GUI_ACTIVE"] / 8 / (d["duration_ms_profiled"] * 1e-3) / 1e9, 3)
json.dump(res, open(dst, "w"), indent=1, sort_keys=True)
for k, d in sorted(res.items()):
    print(k, json.dumps({c: (round(v, 4) if isinstance(v, float) else v) for c, v in sorted(d.items())}))
P
