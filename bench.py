#!/usr/bin/env python3
"""bench.py -- particle-evals/s + tracked FPS of the MI355X PSO hand tracker.

Workload (BASELINE.json configs[1]/[2]): a step is ONE TRACKED FRAME of a synthetic
240x320 depth sequence -- next_frame preprocessing of the raw float32 mm depth (on the
GPU, inside the previous frame's refine launch), refine_init_pose, pso_evolve with 256
particles x 30 generations (reference maxiter = 31), cal_cost(bestp), x0 <- bestp --
the body of test_full's loop (testmodel.cpp:117-139).  The raw frames sit in host
memory, as load_data reads them; --resident prepares them all in HBM first.
N = 250 cloud points (the reference's downsample=true default; --full-cloud: all).

  value        = PSO particle evaluations per second over all ranks
                 (P*(G+1) per frame per rank; refine and final evaluations are not counted)
  tracked_fps  = frames per second (per rank; ranks track the same sequence)
  multi-GPU    = one process per GPU, independent subswarms (seed 1000+rank) with one
                 RCCL all-gather of {bestp, cost} per frame; weak scaling

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1 is launched by torch.distributed.run, one rank per GPU)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "hand-pose-estimation_amd"))

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFLOPS = 157.3  # vector fp32 (spec); the search is fp32 VALU, no MFMA


def algorithmic_bytes_per_eval(n: int) -> int:
    # cloud xyz fp64 (24 B/pt) + 48 x (depth fp64 + DT fp32) gathers
    # + PSO state: read x, v, pbest, pbest[informant]; write x, v, pbest (7 x 26 fp64)
    # + pcost read/write (16 B)                                       
    return 24 * n + 48 * 12 + 7 * 26 * 8 + 16


def algorithmic_flops_per_eval(n: int) -> int:
    # 8 flops per point-sphere pair + 11 per point (alignment)
    # + ~960 (depth) + ~5500 (FK)
    return 8 * 48 * n + 11 * n + 960 + 5500


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--particles", type=int, default=256)
    ap.add_argument("--generations", type=int, default=30)
    ap.add_argument("--full-cloud", action="store_true", help="no down-sampling (N ~ 9.3k)")
    ap.add_argument("--no-refine", action="store_true")
    ap.add_argument("--resident", action="store_true",
                    help="preprocess every frame before timing (default: each step prepares "
                         "the next frame from host depth on the GPU, overlapped)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--seed", type=int, default=0, help="trajectory seed")
    ap.add_argument("--frames", default=os.environ.get("HPE_FRAMES_DIR"),
                    help="directory of MSRA-style *_depth.bin frames (headerless float32 mm, "
                         "240x320) to track instead of the synthetic sequence")
    return ap.parse_args()


def cpu_baseline(args, sizes_hint, recorded=None):
    """The oracle (C restatement, OpenMP over particles where the reference has
    `omp parallel for`) tracking the same synthetic frames on the host: a bounded
    sample of the same workload."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np
    import oracle_c
    import oracle_np
    import hpe
    from hpe import synth
    o = oracle_c.load(build=False)
    d = json.loads((ROOT / "hand-pose-estimation_amd/hpe/hand_subject1.json").read_text())
    geo, rad = np.array(d["hgeo_mm"]) / 10.0, np.array(d["rad_mm"]) / 10.0
    h = o.hand(geo, rad)
    nh = oracle_np.Hand(geo, rad)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    P, G = args.particles, args.generations
    ub, lb, sd = hpe.reference_bounds()
    if recorded is not None:  # the same recorded frames the GPU tracked
        raw = recorded
        poses = [hpe.X0.copy()]
    else:
        poses = synth.trajectory(64, args.seed)
        raw = [oracle_np.render_depth_mm(nh, poses[f]) for f in range(len(poses))]
    x = poses[0].copy()
    done, t0, n_pts = 0, time.perf_counter(), 0
    while True:
        obs = o.preprocess(raw[done % len(raw)], downsample=not args.full_cloud)  # next_frame
        n_pts = obs.n
        if not args.no_refine:
            x, _ = o.refine(h, obs, x)
        x, _, _ = o.pso_evolve(h, obs, x, P, G + 1, lb, ub, sd, seed=1000, nthreads=threads)
        o.cal_cost(h, obs, x)
        done += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or done >= 4096:
            break
    out = {"value": P * (G + 1) * done / el, "unit": "particle-evals/s", "cores": threads,
           "kind": "port", "tracked_fps": done / el,
           "sample": f"{done} tracked frames incl. preprocessing ({P}p x {G} gen, N={n_pts}, "
                     f"refine={'off' if args.no_refine else 'on'}) of the same synthetic "
                     f"sequence in {el:.1f} s, oracle/hpe_oracle.c with {threads} OpenMP threads"}
    # the single-thread rate of the same loop, a shorter sample
    x, done1, t0 = poses[0].copy(), 0, time.perf_counter()
    while True:
        obs = o.preprocess(raw[done1 % len(raw)], downsample=not args.full_cloud)
        if not args.no_refine:
            x, _ = o.refine(h, obs, x)
        x, _, _ = o.pso_evolve(h, obs, x, P, G + 1, lb, ub, sd, seed=1000, nthreads=1)
        o.cal_cost(h, obs, x)
        done1 += 1
        el1 = time.perf_counter() - t0
        if el1 >= args.cpu_seconds / 3 or done1 >= 1024:
            break
    out["one_thread"] = {"value": P * (G + 1) * done1 / el1, "tracked_fps": done1 / el1,
                         "sample": f"{done1} tracked frames in {el1:.1f} s, 1 thread"}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                out["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return out


def load_pmc(P, n_points):
    """HBM traffic per k_pso_gen launch from the committed rocprofv3 --pmc summary."""
    p = ROOT / "profiles" / "pmc_k_pso_gen.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        if d.get("particles") == P and d.get("cloud_points") == n_points:
            return d.get("bytes_per_launch")
    except Exception:
        return None
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with "
                         "torch.distributed.run")
    import numpy as np
    import torch
    import torch.distributed as dist
    import hpe
    from hpe import synth
    from hpe.dist import exchange_best, subswarm_seed

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    P, G = args.particles, args.generations
    hand = hpe.reference_hand(device=local)
    ctx, lib = hand.ctx, hand.ctx.lib
    n_frames = args.warmup + args.steps
    ds = not args.full_cloud
    # the input: raw 240x320 float32 mm depth frames in host memory, as load_data reads
    # them from .bin files (synthetic: rendered once from a seeded pose trajectory)
    if args.frames:  # recorded frames, as load_data reads them (observedmodel.cpp:272-310)
        files = sorted(Path(args.frames).glob("*_depth.bin"))
        if len(files) < n_frames:
            raise SystemExit(f"{args.frames}: {len(files)} *_depth.bin frames, need {n_frames}")
        raw = [np.fromfile(fp, dtype="<f4", count=240 * 320).reshape(240, 320)
               for fp in files[:n_frames]]
        poses = None  # no ground truth: x0 of test_full (testmodel.cpp:38-40)
    else:
        poses = synth.trajectory(n_frames, args.seed)
        raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
    sizes = [len(hpe.preprocess_depth(d, True, ds)["cloud"]) for d in raw]
    NSLOT = 4  # frame slots in rotation: frame f+1 is prepared while frame f is tracked
    slot = (lambda f: f) if args.resident else (lambda f: f % NSLOT)
    if args.resident:  # frames preprocessed and resident in HBM before the timed region
        for f in range(n_frames):
            ctx.prepare_frame(slot(f), raw[f], True, ds)
        ctx.check(lib.hpe_sync(ctx.h))
    ub, lb, sd = hpe.reference_bounds()
    ctx.check(lib.hpe_set_pso_params(ctx.h, hpe._lib.ptr(ub, C.c_double),
                                     hpe._lib.ptr(lb, C.c_double), hpe._lib.ptr(sd, C.c_double),
                                     0.7298, 1.49618, 1.49618, G + 1, 1e-8, 1e-8))
    ctx.check(lib.hpe_set_seed(ctx.h, C.c_uint64(subswarm_seed(rank))))
    state = torch.zeros(27, dtype=torch.float64, device=f"cuda:{local}")
    state[:26] = torch.from_numpy(poses[0] if poses is not None else hpe.X0.copy())
    torch.cuda.synchronize()
    ext = torch.cuda.ExternalStream(lib.hpe_stream(ctx.h), device=f"cuda:{local}")
    gathered = torch.zeros(world * 27, dtype=torch.float64, device=f"cuda:{local}")
    refine = 0 if args.no_refine else 1

    def step(f):
        if args.resident:
            ctx.select_frame(slot(f))
            ctx.check(lib.hpe_track_frame_dev(ctx.h, P, refine, C.c_void_p(state.data_ptr())))
        else:  # frame f tracked while frame f+1 is prepared inside its refine launch
            ctx.track_pipelined(P, refine, state.data_ptr(), raw[f + 1] if f + 1 < n_frames else None)
        if world > 1:  # best-of-N exchange on the tracker's own stream (no host sync)
            with torch.cuda.stream(ext):
                exchange_best(state, gathered)

    if not args.resident:
        ctx.pipeline_begin(raw[0], True, ds)
    for f in range(args.warmup):
        step(f)
    ctx.check(lib.hpe_sync(ctx.h))
    torch.cuda.synchronize()
    # timed region: graph-replayed frames, nothing else on the tracker stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_s = 0.0
    for f in range(args.warmup, n_frames):
        h0 = time.perf_counter()
        step(f)
        host_s += time.perf_counter() - h0
    ctx.check(lib.hpe_sync(ctx.h))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    final = state.cpu().numpy()
    # per-frame device time: the same frames again with one event pair per frame on the
    # tracker stream (not in the timed region: each timing event adds a marker, ~5 us)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if not args.resident:
        ctx.pipeline_begin(raw[args.warmup], True, ds)
    for k, f in enumerate(range(args.warmup, n_frames)):
        ev[k][0].record(ext)
        step(f)
        ev[k][1].record(ext)
    ctx.check(lib.hpe_sync(ctx.h))
    torch.cuda.synchronize()
    frame_us = [a.elapsed_time(b) * 1e3 for a, b in ev]
    # per-kernel durations: the same frames once more with every dispatch bracketed by
    # hipExtLaunchKernel start/stop events (direct launches; kernels are identical)
    ctx.check(lib.hpe_profile_enable(ctx.h, 1))
    if not args.resident:
        ctx.pipeline_begin(raw[args.warmup], True, ds)
    errs = []  # gnd_truth_err (costfunc.cpp:476-507) of each frame's bestp vs the true pose
    for f in range(args.warmup, n_frames):
        step(f)
        ctx.check(lib.hpe_sync(ctx.h))
        torch.cuda.synchronize()
        if poses is None:
            continue
        bp = state[:26].cpu().numpy()
        hand.build_hand_model(bp)
        est = hand.hand_joints.copy()
        hand.build_hand_model(poses[f])
        gt = hand.hand_joints * 10.0
        gt[:, 1:3] *= -1
        errs.append(hpe.gnd_truth_err(est, gt.ravel()))
    ctx.check(lib.hpe_sync(ctx.h))
    prof = {}
    for name, kid in (("k_pso_gen", 0), ("k_refine", 1), ("k_pso_init", 2), ("k_pso_final", 3),
                      ("k_preprocess", 4)):
        nl = C.c_int32(0); tot = C.c_double(0); mn = C.c_double(0); mx = C.c_double(0)
        ctx.check(lib.hpe_profile_read_kernel(ctx.h, kid, C.byref(nl), C.byref(tot),
                                              C.byref(mn), C.byref(mx)))
        prof[name] = {"launches": nl.value, "avg_us": tot.value / max(nl.value, 1) * 1e3,
                      "min_us": mn.value * 1e3, "max_us": mx.value * 1e3,
                      "total_ms": tot.value}
    ctx.check(lib.hpe_profile_enable(ctx.h, 0))
    prof["frame_graph"] = {"launches": len(frame_us), "avg_us": sum(frame_us) / len(frame_us),
                           "min_us": min(frame_us), "max_us": max(frame_us),
                           "note": "one event pair per frame, a second pass over the frames"}

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    n_pts = sizes[args.warmup]
    evals = P * (G + 1) * args.steps * world
    pg = prof["k_pso_gen"]
    avg_s = pg["avg_us"] * 1e-6
    bytes_launch = P * algorithmic_bytes_per_eval(n_pts)
    flops_launch = P * algorithmic_flops_per_eval(n_pts)
    achieved = bytes_launch / avg_s / 1e9 if pg["launches"] else None
    valu = flops_launch / avg_s / 1e12 if pg["launches"] else None
    line = {
        "metric": "particle-evals/sec + tracked FPS, 320x240 depth, 256p x 30gen",
        "value": evals / el,
        "unit": "particle-evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32+f64",
        "data": (f"recorded: {n_frames} *_depth.bin frames from {args.frames}" if args.frames else
                 "synthetic: seeded 26-DOF trajectory rendered from the 48-sphere model "
                 "into 240x320 float32 mm depth (no MSRA Subject1 on the box)"),
        "config": {"workload": ("tracked frame = " + ("" if args.resident else
                                "next_frame preprocessing (GPU, fused into the refine launch) + ") +
                                "refine_init_pose + pso_evolve + cal_cost(bestp)"),
                   "particles": P, "generations": G, "maxiter": G + 1,
                   "cloud_points": n_pts, "refine": bool(refine),
                   "parallelism": f"subswarms x{world}, all-gather best per frame"},
        "tracked_fps": args.steps / el,
        "final_cost": float(final[26]),
        "tracking_err_mm": ({"sum_wrist_tips_mean": float(np.mean(errs)),
                             "per_joint_mean": float(np.mean(errs) / 6),
                             "note": "gnd_truth_err (costfunc.cpp:476-507) vs the synthetic "
                                     "trajectory's true poses, second pass over the frames"}
                            if errs else None),
        "roofline": {
            "bound": "hbm", "kernel": "k_pso_gen",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None,
            "traffic": load_pmc(P, n_pts),
            "avg_launch_us": pg["avg_us"], "launches": pg["launches"],
            "bytes_per_launch": bytes_launch,
            "flops_per_launch": flops_launch,
            "valu_tflops": valu,
            "valu_frac": valu / FP32_PEAK_TFLOPS if valu else None,
            "note": "algorithmic bytes per launch = P*(24N + 2048), per-launch time from "
                    "hipExtLaunchKernel events on the tracker stream; the generation is "
                    "latency-bound (one particle per workgroup, 31 dependent launches per "
                    "frame), DESIGN.md §5"},
        "kernels": prof,
        "host_us_per_step": host_s / args.steps * 1e6,
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args, sizes, raw if args.frames else None)
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
