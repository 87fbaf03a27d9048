#!/usr/bin/env python3
"""Benchmark: mantis3 rig poses/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], the metric's "1280x720 4-cam batch"): rigs
of 4 fisheye cameras at 1280x720 over the IARC-style grid, shared map
(params/map.yaml, 720 landmarks); the full reference per-camera path
(detector -> RPP -> clustering -> scoring -> particle filter -> shifts ->
yaw -> publish gate) plus the rig fusion, batched `--rigs` rigs per step.
A step = one mantis_process_batch over the batch; frames are synthetic,
rendered once into HBM before timing (inputs resident in HBM).

Multi-GPU: one process per GPU (torchrun); rigs are independent units, each
rank processes its own batch (weak scaling, no collective on the data path);
barrier + device sync bracket the timed region and the max time over ranks is
reported. value = rig poses/s of the whole job.

Also reported: p50 single-rig latency (host submit -> result), the dominant
kernel's roofline (HIP events on the library stream during the timed region)
and the CPU oracle baseline timed on this host (rank 0, N=1 only).
"""
import argparse
import ctypes as C
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector spec
# FP64 operations of one ObjPose iteration (one AbsKernel: the 3x3 accumulations,
# OpenCV's one-sided Jacobi SVD, R, t and the error), counted by
# tools/rpp_flops.cpp on the host build of mk_rpp.h (+,-,*,/,sqrt,hypot = 1 each).
# 1704 = what the device executes: the Jacobi noise-phase fast-forward
# (mk_rpp.h jacobi_noise_ff) skips the ~19 sweeps that only shrink the
# rank-deficient row (the full reference sweep count is 4282 per iteration).
FLOPS_PER_OBJPOSE_ITER = 1704
W, H = 1280, 720
CAMS = 4
LANDMARKS = 720
FLOPS_PER_PROJ = 51         # BASELINE.md roofline formulas
FLOPS_PER_WINDOW = 200


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rigs", type=int, default=3072, help="rigs per step per GPU")
    p.add_argument("--distinct", type=int, default=16, help="distinct rendered rigs (cycled)")
    p.add_argument("--contexts", type=int, default=3,
                   help="library contexts per GPU, each driven by its own host thread (one ctx per thread, "
                        "include/mantis.h); the step's rigs are split evenly between them")
    p.add_argument("--latency-iters", type=int, default=15)
    p.add_argument("--cpu-rigs", type=int, default=6, help="rigs timed on the CPU oracle (bounded sample)")
    p.add_argument("--hw-queues", type=int, default=4,
                   help="GPU_MAX_HW_QUEUES for this process, so the contexts' streams run on separate hardware queues")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--gn", type=int, default=1,
                   help="joint rig Gauss-Newton after the per-camera pipeline (SURVEY §8 d config 3); 0 = reference-parity only")
    p.add_argument("--gn-iterations", type=int, default=8)
    p.add_argument("--max-contour-points", type=int, default=98304,
                   help="per-frame contour point pool (720p frames use ~22k, max seen 28k; overflow is reported as an error)")
    return p.parse_args()


def main():
    a = parse()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(max(4, min(32, a.hw_queues))))  # before HIP initialises
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist

        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        tdist.init_process_group(backend=backend)
        dist = tdist

    import mantis_amd as M
    from mantis_amd import synth

    white, red, green = synth.load_map()
    K, D = synth.intrinsics(W, H)
    n_frames = a.rigs * CAMS
    nctx = max(1, min(a.contexts, a.rigs))
    assert a.rigs % nctx == 0, "--rigs must be a multiple of --contexts"
    rigs_ctx = a.rigs // nctx
    ctxs = []
    for _ in range(nctx):
        mc = M.Mantis(M.default_config(device=local, max_cams=rigs_ctx * CAMS, max_width=W, max_height=H,
                                       gn_enable=a.gn, gn_iterations=a.gn_iterations,
                                       max_contour_points=a.max_contour_points))
        mc.set_map(white, red, green)
        ctxs.append(mc)
    m = ctxs[0]

    # ---- synthetic rigs rendered into HBM once
    rng = np.random.default_rng(1000 + rank)
    ext = synth.rig_extrinsics(CAMS)
    cams, Tbc = [], []
    for r in range(a.distinct):
        Twb = synth.random_base_pose(rng)
        for c in range(CAMS):
            Twc = Twb @ ext[c]
            cams.append(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H))
            Tbc.append(ext[c])
    nd = len(cams)
    fb = W * H * 3
    dev = m.device_alloc(nd * fb)
    seeds = [synth.frame_seed(3, i + 100000 * rank) for i in range(nd)]
    m.synth_render(cams, seeds, dev)
    m.synchronize()
    imgs = []
    for i in range(n_frames):
        j = i % nd
        imgs.append(M.make_image(None, K, D, T_base_cam=Tbc[j], device_ptr=dev + j * fb, width=W, height=H))
    per_ctx = [imgs[k * rigs_ctx * CAMS:(k + 1) * rigs_ctx * CAMS] for k in range(nctx)]
    from concurrent.futures import ThreadPoolExecutor

    pool = ThreadPoolExecutor(max_workers=nctx)

    def run_step():
        """One step: every context processes its share of the rigs, concurrently."""
        futs = [pool.submit(ctxs[k].process, per_ctx[k], rigs_ctx) for k in range(nctx)]
        outs = [f.result() for f in futs]
        rig = [r for o in outs for r in o[0]]
        cam = [c for o in outs for c in o[1]]
        return rig, cam

    def barrier_sync():
        if dist is not None:
            dist.barrier()
        for mc in ctxs:
            mc.synchronize()

    # ---- warmup
    for _ in range(a.warmup):
        run_step()

    # ---- timed region: stage events on the library stream
    m.set_profiling(True)
    stage_ms = {}
    scored = 0
    published = 0
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        rig, cam = run_step()
        for name, ms in m.kernel_times():
            stage_ms[name] = stage_ms.get(name, 0.0) + ms
        scored += sum(c.n_scored for c in cam)
        published += sum(r.publish for r in rig)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    m.set_profiling(False)
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        if torch.cuda.is_available():
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    poses = a.rigs * a.steps * world
    value = poses / elapsed
    ms_per_step = elapsed / a.steps * 1e3

    # ---- per-step work counts (every step processes the same frames, so the
    # counters of the last step describe each step): ObjPose iterations of the
    # two RPP queues, scored hypotheses
    frames_step = rigs_ctx * CAMS  # stage events are recorded on context 0's stream, over its frames
    iters = [0, 0]
    for i in range(frames_step):
        fc = m.frame_counters(i)
        iters[0] += int(fc[16])
        iters[1] += int(fc[17])
    scored_per_frame = scored / max(1, a.steps * n_frames)
    slow_per_frame = 80.0
    fast_per_frame = max(0.0, scored_per_frame - slow_per_frame)
    s_fast = LANDMARKS * fast_per_frame
    s_slow = 3700.0 * slow_per_frame

    # ---- roofline of the dominant stage (per launch = per step on context 0)
    avg = {k: v / a.steps for k, v in stage_ms.items()}
    # algorithmic bytes (HBM-bound stages) or FP64 flops (VALU-bound stages) per launch
    work = {
        # BGR read once; candidate and strong-root bit planes written
        "canny_nms": ("hbm", frames_step * (3 * W * H + W * H // 4)),
        # candidate bits read, edge bits written
        "hysteresis": ("hbm", frames_step * (W * H // 4)),
        # edge bits read once; padded detector bits and mask bits written
        "morph": ("hbm", frames_step * (W * H // 8 + (W + 2) * (H + 2) // 8 + W * H // 8)),
        "components": ("hbm", frames_step * (5 * (W + 2) * (H + 2))),
        "border_trace": ("hbm", frames_step * ((W + 2) * (H + 2) // 8)),
        "contours_quads": ("hbm", frames_step * ((W + 2) * (H + 2) // 8)),
        "rpp_first": ("fp64", iters[0] * FLOPS_PER_OBJPOSE_ITER),
        "rpp_cand": ("fp64", iters[1] * FLOPS_PER_OBJPOSE_ITER),

        "score_pf_yaw": ("fp64", frames_step * (FLOPS_PER_PROJ * (s_fast + 37 * slow_per_frame) +
                                                FLOPS_PER_WINDOW * 37 * slow_per_frame)),
    }

    def roofline(stage, avg=avg):
        if stage not in avg or stage not in work:
            return None
        kind, amount = work[stage]
        dur_s = avg[stage] * 1e-3
        if kind == "hbm":
            achieved = amount / dur_s / 1e9
            traffic = None
            pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                try:
                    tj = json.load(open(pmc))
                    if tj.get("stage") == stage and tj.get("hbm_bytes_per_frame"):
                        traffic = int(tj["hbm_bytes_per_frame"] * frames_step)
                except Exception:
                    traffic = None
            return {"bound": "hbm", "kernel": stage, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "alg_bytes_per_launch": int(amount), "avg_launch_ms": round(avg[stage], 4)}
        achieved = amount / dur_s / 1e12
        return {"bound": "fp64_valu", "kernel": stage, "achieved": round(achieved, 4), "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 5), "traffic": None,
                "alg_flops_per_launch": int(amount), "avg_launch_ms": round(avg[stage], 4)}

    kern = [k for k in avg if k in work]
    dom = max(kern, key=avg.get) if kern else None  # dominant kernel stage by event time
    roof = roofline(dom) if dom else None
    if roof is not None:
        roof["stages_ms"] = {k: round(v, 4) for k, v in sorted(avg.items(), key=lambda kv: -kv[1])}
        roof["objpose_iterations_per_launch"] = iters
    roof_front = roofline("canny_nms")

    # ---- the same stages with context 0 running alone (one step, after the
    # timed region): the timed-region launch durations above include the
    # other contexts' kernels sharing the CUs; these are the kernels' own
    if nctx > 1 and roof is not None:
        m.set_profiling(True)
        ctxs[0].process(per_ctx[0], rigs_ctx)
        iso = {k: v for k, v in m.kernel_times()}
        m.set_profiling(False)
        for r, stg in ((roof, dom), (roof_front, "canny_nms")):
            ri = roofline(stg, iso) if r is not None else None
            if ri is not None:
                r["isolated"] = {"avg_launch_ms": ri["avg_launch_ms"], "achieved": ri["achieved"], "frac": ri["frac"],
                                 "note": "context 0 alone, one step after the timed region"}
        roof["stages_ms_isolated"] = {k: round(v, 4) for k, v in sorted(iso.items(), key=lambda kv: -kv[1])}
    path_bytes = n_frames * (6 * W * H + 3 * (s_fast + s_slow))

    # ---- p50 latency of one rig (host submit -> result on host)
    lat = []
    one = imgs[:CAMS]
    for _ in range(a.latency_iters):
        t1 = time.perf_counter()
        m.process(one, rigs=1)
        lat.append(time.perf_counter() - t1)
    p50 = float(np.median(lat)) * 1e3

    # ---- CPU baseline: the oracle (C++ -O2 restatement) on a bounded sample, 1 core
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        try:
            import _oracle as O

            orc = O.Oracle(white, red, green, seed=1)
            host = [np.zeros((H, W, 3), np.uint8) for _ in range(a.cpu_rigs * CAMS)]
            for i in range(len(host)):
                m.d2h(host[i], dev + (i % nd) * fb)
            t1 = time.perf_counter()
            for i in range(len(host)):
                orc.process(host[i], K, D)
            dt = time.perf_counter() - t1
            cpu = {"value": round(a.cpu_rigs / dt, 4), "unit": "rig poses/s", "cores": 1, "kind": "port",
                   "sample": f"{a.cpu_rigs} rigs x {CAMS} cams 1280x720 through oracle/liboracle.so "
                             f"(full mantis3 callback per camera), {dt:.1f} s on 1 host core"}
        except Exception as e:  # the oracle is optional on a box without it
            cpu = {"value": None, "unit": "rig poses/s", "cores": 1, "kind": "port", "sample": f"unavailable: {e}"}

    if rank == 0:
        line = {
            "metric": "poses/sec + p50 per-frame latency, 1280x720 4-cam batch",
            "value": round(value, 3), "unit": "rig poses/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic fisheye grid frames rendered in HBM (SURVEY §8d scene), map.yaml landmarks",
            "config": {"workload": "config3: 4-cam 1280x720 rig, shared map, full mantis3 path per camera"
                                    + (" + joint rig Gauss-Newton" if a.gn else ""),
                       "rigs_per_step_per_gpu": a.rigs, "cams_per_rig": CAMS, "frames_per_step_per_gpu": n_frames,
                       "contexts_per_gpu": nctx,
                       "resolution": [W, H], "landmarks": LANDMARKS, "parallelism": f"rig-data-parallel x{world}"},
            "p50_latency_ms": round(p50, 3),
            "camera_frames_per_s": round(value * CAMS, 2),
            "published_frac": round(published / max(1, a.rigs * a.steps), 4),
            "path_alg_GBps": round(path_bytes * a.steps / elapsed / 1e9, 3),
            "roofline": roof,
            "roofline_frontend": roof_front,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    pool.shutdown()
    for mc in ctxs:
        mc.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
