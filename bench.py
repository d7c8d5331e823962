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
                 RCCL all-gather of {bestp, cost} per frame; weak scaling.
                 --exchange-form library (default with nccl): libhpe.so's own communicator
                 (hpe_subswarm_init), the exchange captured into the 8-frame graphs, so N
                 ranks run the N = 1 loop; torch: torch.distributed per frame, one graph per
                 frame (and the gloo rehearsal)

--config selects a BASELINE.json workload: seq (default; configs[1]/[2]: 256 x 30 tracked
frames), p32 (configs[0]'s shape, 32 x 10), p4096 (configs[3], 4096 x 40), subswarm8
(configs[4]: 1024 particles per rank x 30; run with --gpus 8).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]
       --gpus N > 1 without a torch.distributed environment re-launches itself under
       `python -m torch.distributed.run --nproc-per-node N` (a child process started
       before anything touches the GPU) and exits with its return code.
       --stub: no GPU -- each rank exchanges a stub tracker state over gloo (CPU test of
       the launcher and the exchange).
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "hand-pose-estimation_amd"))

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
# the synthetic sequence: trajectory seed and mean reversion toward x0 (keeps the hand in
# view); fixed from round 2 on so bench lines compare round over round
TRAJ_SEED, TRAJ_REVERT = 0, 0.02
FP32_PEAK_TFLOPS = 157.3  # vector fp32 (spec); the search is fp32 VALU, no MFMA

CONFIGS = {  # name -> (particles, generations, BASELINE.json workload)
    "seq": (256, 30, "configs[1]/[2]: tracked sequence, 256 particles x 30 generations, "
                     "refine + temporal prior"),
    "p32": (32, 10, "configs[0]'s shape on the GPU: 32 particles x 10 generations"),
    "p4096": (4096, 40, "configs[3]: large swarm, 4096 particles x 40 generations"),
    "subswarm8": (1024, 30, "configs[4]: 1024-particle subswarm per rank x 30 generations, "
                            "all-gather of the best per frame"),
}


def algorithmic_bytes_per_eval(n: int) -> int:
    # SURVEY.md §8 d2 / BASELINE.md §3: fp32 xyz cloud (12 B/pt) + 48 x (depth + DT)
    # gathers (384 B) + theta (208 B) + cost (8 B) = 12N + 600
    return 12 * n + 600


def algorithmic_flops_per_eval(n: int) -> int:
    # 8 flops per point-sphere pair + 11 per point (alignment)
    # + ~960 (depth) + ~5500 (FK)
    return 8 * 48 * n + 11 * n + 960 + 5500


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="seq")
    ap.add_argument("--particles", type=int, default=None, help="override the config's P")
    ap.add_argument("--generations", type=int, default=None, help="override the config's G")
    ap.add_argument("--full-cloud", action="store_true", help="no down-sampling (N ~ 9.3k)")
    ap.add_argument("--no-refine", action="store_true")
    ap.add_argument("--resident", action="store_true",
                    help="preprocess every frame before timing (default: each step prepares "
                         "the next frame from host depth on the GPU, overlapped)")
    ap.add_argument("--frames-per-graph", type=int, default=None,
                    help="frames captured per graph launch: the raw depth frames resident in "
                         "HBM, each next frame prepared inside the previous frame's refine "
                         "launch (hpe_track_raw_sequence_dev); with --resident the prepared "
                         "frames through hpe_track_sequence_dev.  0: one graph per frame "
                         "(hpe_track_pipelined from host frames / hpe_track_frame_dev).  "
                         "Default: 8 (one GPU, or N > 1 with the library exchange), 0 with "
                         "--exchange-form torch / gloo, --dump or --exchange gen:K")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=TRAJ_SEED, help="trajectory seed")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process group for --gpus N > 1 (nccl = RCCL over xGMI; gloo: the "
                         "per-frame exchange through host memory, a rehearsal mode)")
    ap.add_argument("--exchange", default="frame",
                    help="frame (default): the ranks' best is exchanged once per tracked frame "
                         "(the reference's best-of-N, SURVEY.md §8e); gen:K additionally "
                         "exchanges every K generations and injects the global best as an "
                         "extra informant (ICP-PSO style, NOT the reference algorithm)")
    ap.add_argument("--exchange-form", choices=("library", "torch"), default=None,
                    help="N > 1: library (default with nccl) = libhpe.so's RCCL all-gather + "
                         "pick after every frame, captured in the frame graphs "
                         "(hpe_subswarm_init); torch = torch.distributed all_gather per frame "
                         "between one-frame graphs (gloo always)")
    ap.add_argument("--subswarm-world1", action="store_true",
                    help="--gpus 1: run the library exchange on a one-rank RCCL communicator "
                         "(the N > 1 loop's cost at N = 1; VERDICT r5 item 1)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank uses cuda:0 (rehearse N ranks on a one-GPU box; with "
                         "--backend gloo)")
    ap.add_argument("--frames", default=os.environ.get("HPE_FRAMES_DIR"),
                    help="directory of MSRA-style *_depth.bin frames (headerless float32 mm, "
                         "240x320) to track instead of the synthetic sequence")
    ap.add_argument("--dump", default=None,
                    help="test mode: each rank saves its state after every frame of the first "
                         "pass (synchronising per frame) and rank 0 the first raw frame and x0, "
                         "as .npy under this directory")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.exchange_form is None:
        a.exchange_form = "library" if a.backend == "nccl" and a.exchange == "frame" else "torch"
    if a.exchange_form == "library" and a.backend != "nccl":
        ap.error("--exchange-form library needs --backend nccl (RCCL)")
    if a.subswarm_world1 and a.gpus != 1:
        ap.error("--subswarm-world1 is the one-GPU rehearsal of the library exchange")
    # the library exchange sits inside the frames' graphs: N ranks run the N = 1 loop
    a.lib_exchange = (a.gpus > 1 and a.exchange_form == "library") or a.subswarm_world1
    graphs_ok = (a.gpus == 1 or a.lib_exchange) and not a.dump
    if a.frames_per_graph is None:
        a.frames_per_graph = 8 if (graphs_ok and a.exchange == "frame") else 0
    if a.frames_per_graph and not graphs_ok:
        ap.error("--frames-per-graph needs one GPU or the library exchange, and no --dump "
                 "(a per-frame torch exchange / dump sits between frames)")
    a.exchange_every = 0
    if a.exchange != "frame":
        if not a.exchange.startswith("gen:") or not a.exchange[4:].isdigit() or int(a.exchange[4:]) < 1:
            ap.error("--exchange takes frame or gen:K with K >= 1")
        a.exchange_every = int(a.exchange[4:])
        if a.frames_per_graph:
            ap.error("--exchange gen:K runs without graph replay (no --frames-per-graph)")
    P, G, _ = CONFIGS[a.config]
    a.particles = a.particles or P
    a.generations = a.generations if a.generations is not None else G
    return a


# ------------------------------------------------------------------------- extra passes
def extra_passes(args, ctx, lib, state, state0, raw, n_frames, P, refine, ds, world, rank, local):
    """Diagnostic passes over the timed frames, after the timed region (never in `value`):
      refine_exact_ms_per_step   the same loop with the reference-order refine (DH chain on
                                 every evaluation, hpe_set_refine_exact(1))
      per_frame_graph_ms_per_step (N = 1) the per-frame pipelined loop (one graph per frame, raw
                                 frames from host memory: the PCIe-inclusive form, and the loop
                                 of `--exchange-form torch` lines)
      scaling_baseline_ms_per_step (N > 1) every rank tracks the frames alone, no exchange, in
                                 the timed loop's form (the library exchange suspended:
                                 hpe_subswarm_enable(0); the torch form: the per-frame loop);
                                 the max over ranks: the N = 1 figure of this loop on these GPUs
      exchange_off_ms_per_step   (--subswarm-world1) the timed loop with the library exchange
                                 suspended: the plain N = 1 loop in the same run
    Each pass runs the frames twice (graph captures in the first) and times the second."""
    import numpy as np
    import torch
    import torch.distributed as dist

    exact0 = int(lib.hpe_get_refine_exact(ctx.h))
    out = {"refine_form": ("chain: the reference's DH chain on every evaluation" if exact0 else
                           "hand-frame: spheres Rg q + u from centres built once per call, FK "
                           "within 1e-12 cm of the chain (DESIGN.md §2)"),
           "refine_kernel": "k_refine, one workgroup",
           "refine_exact_ms_per_step": None, "per_frame_graph_ms_per_step": None,
           "scaling_baseline_ms_per_step": None, "exchange_off_ms_per_step": None,
           "note": ("diagnostic passes after the timed region over the same frames (second of two "
                    "runs each): refine_exact = reference-order refine; per_frame_graph = one "
                    "graph per frame from host memory (PCIe-inclusive; the torch-exchange loop); "
                    "scaling_baseline (N > 1) = the timed loop on every rank alone, exchange "
                    "suspended, max over ranks; exchange_off (--subswarm-world1) = the timed loop "
                    "with the exchange suspended")}
    if not refine:
        return out
    d_raw = None

    def run(K2):
        nonlocal d_raw
        state.copy_(state0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if K2 and args.resident:  # the timed loop's form: prepared frames
            ctx.track_sequence(P, refine, state.data_ptr(), args.warmup, args.steps, K2)
        elif K2:
            if d_raw is None:
                d_raw = torch.from_numpy(np.ascontiguousarray(np.stack(raw), dtype=np.float32)).to(
                    f"cuda:{local}")
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            ctx.track_raw_sequence(P, refine, state.data_ptr(),
                                   d_raw.data_ptr() + args.warmup * d_raw[0].numel() * 4, args.steps,
                                   True, ds, frames_per_graph=K2)
        else:
            ctx.pipeline_begin(raw[args.warmup], True, ds)
            for f in range(args.warmup, n_frames):
                ctx.track_pipelined(P, refine, state.data_ptr(), raw[f + 1] if f + 1 < n_frames else None)
        ctx.check(lib.hpe_sync(ctx.h))
        return (time.perf_counter() - t0) / args.steps * 1e3

    def twice(K2):
        run(K2)
        return run(K2)

    K = args.frames_per_graph
    if world == 1 and args.lib_exchange:  # the same loop, the exchange suspended
        ctx.subswarm_enable(False)
        out["exchange_off_ms_per_step"] = twice(K)
        ctx.subswarm_enable(True)
    ctx.check(lib.hpe_set_refine_exact(ctx.h, 1))
    out["refine_exact_ms_per_step"] = twice(K) if world == 1 else None
    ctx.check(lib.hpe_set_refine_exact(ctx.h, exact0))
    if world == 1:
        out["per_frame_graph_ms_per_step"] = twice(0)
    else:
        if args.lib_exchange:
            ctx.subswarm_enable(False)
        ms = torch.tensor([twice(K if args.lib_exchange else 0)], dtype=torch.float64)
        if args.lib_exchange:
            ctx.subswarm_enable(True)
        if args.backend == "nccl":
            ms = ms.to(f"cuda:{local}")
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        out["scaling_baseline_ms_per_step"] = float(ms.cpu()[0])
    state.copy_(state0)
    torch.cuda.synchronize()
    return out


# ------------------------------------------------------------------------- launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(args) -> int:
    """--gpus N > 1 from a plain invocation: run this script under torch.distributed.run
    as a child process (nothing in this process has touched the GPU), relay its output,
    return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


# ------------------------------------------------------------------------- CPU baseline
def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 cpu.max quota (None: unlimited or unknown)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(round(int(q) / int(per))))
    except (OSError, ValueError):
        return None


def cpu_baseline(args, recorded=None):
    """The oracle (C restatement, OpenMP over particles where the reference has
    `omp parallel for`, PSO.cpp:748,848) tracking the same synthetic frames on the host:
    bounded samples of the same workload.  Threads: the reference's OpenMP default, every
    CPU of the process's affinity (nproc); also at the cgroup CPU quota
    when one is set below it (oversubscribed OpenMP barriers stall); the faster leg is
    the reported value.  Plus a 1-thread leg."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_c
    import oracle_np
    import hpe
    from hpe import synth
    o = oracle_c.load(build=False)
    d = json.loads((ROOT / "hand-pose-estimation_amd/hpe/hand_subject1.json").read_text())
    geo, rad = d["hgeo_mm"], d["rad_mm"]
    import numpy as np
    geo, rad = np.array(geo) / 10.0, np.array(rad) / 10.0
    h = o.hand(geo, rad)
    nh = oracle_np.Hand(geo, rad)
    P, G = args.particles, args.generations
    ub, lb, sd = hpe.reference_bounds()
    if recorded is not None:  # the same recorded frames the GPU tracked
        raw, x_start = recorded, hpe.X0.copy()
    else:
        poses = synth.trajectory(64, args.seed, revert=TRAJ_REVERT)
        raw = [oracle_np.render_depth_mm(nh, poses[f]) for f in range(len(poses))]
        x_start = poses[0].copy()

    def leg(threads, seconds, max_frames):
        x, done, t0, n_pts = x_start.copy(), 0, time.perf_counter(), 0
        while True:
            obs = o.preprocess(raw[done % len(raw)], downsample=not args.full_cloud)
            n_pts = obs.n
            if not args.no_refine:
                x, _ = o.refine(h, obs, x)
            x, _, _ = o.pso_evolve(h, obs, x, P, G + 1, lb, ub, sd, seed=1000, nthreads=threads)
            o.cal_cost(h, obs, x)
            done += 1
            el = time.perf_counter() - t0
            if el >= seconds or done >= max_frames:
                return {"value": P * (G + 1) * done / el, "tracked_fps": done / el,
                        "threads": threads, "frames": done, "seconds": el, "cloud_points": n_pts}

    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    skipped = None
    if quota and quota < affinity:
        # more OpenMP threads than the cgroup grants stall at every barrier (measured on
        # the box: 256 affinity threads under a 16-CPU quota ran 0.26 FPS): time the quota
        legs = {"cgroup_quota": leg(quota, args.cpu_seconds, 4096)}
        skipped = (f"affinity leg ({affinity} threads) not run: the cgroup quota grants "
                   f"{quota} CPUs, so {affinity} OpenMP threads would be oversubscribed")
    else:
        legs = {"affinity": leg(affinity, args.cpu_seconds, 4096)}
    best = max(legs.values(), key=lambda r: r["value"])
    one = leg(1, args.cpu_seconds / 3, 1024)
    out = {"value": best["value"], "unit": "particle-evals/s", "cores": best["threads"],
           "kind": "port", "tracked_fps": best["tracked_fps"],
           "sample": (f"{best['frames']} tracked frames incl. preprocessing ({P}p x {G} gen, "
                      f"N={best['cloud_points']}, refine={'off' if args.no_refine else 'on'}) "
                      f"of the same synthetic sequence in {best['seconds']:.1f} s, "
                      f"oracle/hpe_oracle.c with {best['threads']} OpenMP threads"),
           "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "skipped_leg": skipped,
           "legs": {k: {kk: v[kk] for kk in ("threads", "value", "tracked_fps", "frames")}
                    for k, v in legs.items()},
           "one_thread": {"value": one["value"], "tracked_fps": one["tracked_fps"],
                          "sample": f"{one['frames']} tracked frames in {one['seconds']:.1f} s, "
                                    f"1 thread"}}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                out["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return out


# ------------------------------------------------------------------------- roofline
def lib_sha256(path):
    return hashlib.sha256(Path(path).read_bytes()).hexdigest()


def load_pmc(kernel, P, n_points, lib_path):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary
    (profiles/pmc_<kernel>.json), only if it was captured from this very libhpe.so build
    and workload; otherwise None."""
    p = ROOT / "profiles" / f"pmc_{kernel}.json"
    if not p.exists():
        return None, "no PMC capture committed"
    try:
        d = json.loads(p.read_text())
    except ValueError:
        return None, "unreadable PMC capture"
    if d.get("lib_sha256") != lib_sha256(lib_path):
        return None, "PMC capture is of another libhpe.so build"
    if d.get("particles") != P or d.get("cloud_points") != n_points:
        return None, "PMC capture is of another workload"
    return d.get("bytes_per_launch"), f"profiles/pmc_{kernel}.json (same build, sha256 match)"


def roofline_entry(kernel, prof, evals_per_launch, n_pts, lib_path, P):
    k = prof[kernel]
    if not k["launches"]:
        return None
    avg_s = k["avg_us"] * 1e-6
    bpl = evals_per_launch * algorithmic_bytes_per_eval(n_pts)
    fpl = evals_per_launch * algorithmic_flops_per_eval(n_pts)
    achieved = bpl / avg_s / 1e9
    traffic, tsrc = load_pmc(kernel, P, n_pts, lib_path)
    valu = fpl / avg_s / 1e12
    return {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_source": tsrc, "avg_launch_us": k["avg_us"], "launches": k["launches"],
            "evals_per_launch": evals_per_launch, "bytes_per_launch": bpl,
            "flops_per_launch": fpl, "valu_tflops": valu, "valu_frac": valu / FP32_PEAK_TFLOPS}


# ------------------------------------------------------------------------- stub ranks
def device_identity(local):
    """This rank's GPU: PCI domain:bus:device and UUID from the HIP device properties."""
    import torch
    pr = torch.cuda.get_device_properties(local)
    pci = ":".join(str(getattr(pr, k, "?")) for k in ("pci_domain_id", "pci_bus_id",
                                                        "pci_device_id"))
    return {"pci": pci, "uuid": str(getattr(pr, "uuid", "")), "name": pr.name,
            "local_rank": local}


def rccl_version():
    import torch
    try:
        v = torch.cuda.nccl.version()
        return ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception as e:  # noqa: BLE001
        return f"unavailable ({type(e).__name__})"


def rank_report(args, world, rank, el, final, dev, ident):
    """Self-verification of a multi-rank run (every rank calls it): the world size from the
    process group, the collective library's version, each rank's device (distinct unless
    --same-device), min / max of the ranks' times, and every rank's final 27-double state
    identical (all adopted the same best at the last exchange).  Returns (max time over
    ranks, the report); raises SystemExit on a failed check."""
    import numpy as np
    import torch
    import torch.distributed as dist
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    ts = torch.zeros(world, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(ts, t)
    el_all = ts.cpu().numpy()
    fs = torch.from_numpy(np.ascontiguousarray(final, dtype=np.float64)).to(dev)
    fa = torch.zeros(world * 27, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(fa, fs)
    fa = fa.cpu().numpy().reshape(world, 27)
    same_state = bool(np.all((fa == fa[0]) | (np.isnan(fa) & np.isnan(fa[0]))))
    ids = [None] * world
    dist.all_gather_object(ids, ident)
    keys = [d["pci"] + "/" + d["uuid"] for d in ids]
    distinct = len(set(keys)) == world
    rep = {"world_size_pg": dist.get_world_size(), "backend": dist.get_backend(),
           "rccl_version": rccl_version() if dist.get_backend() == "nccl" else None,
           "devices": ids, "devices_distinct": distinct,
           "same_device_mode": bool(args.same_device),
           "ms_per_step_min": float(el_all.min()) / args.steps * 1e3,
           "ms_per_step_max": float(el_all.max()) / args.steps * 1e3,
           "final_state_identical": same_state}
    if rep["world_size_pg"] != world:
        raise SystemExit(f"rank {rank}: process group of {rep['world_size_pg']}, WORLD_SIZE {world}")
    if not same_state:
        raise SystemExit(f"rank {rank}: the ranks' final states differ after the exchange")
    if not distinct and not args.same_device:
        raise SystemExit(f"rank {rank}: two ranks share a device ({keys}); --same-device "
                         "rehearses several ranks on one GPU")
    return float(el_all.max()), rep


def stub_main(args, world, rank):
    """CPU rehearsal of the multi-rank path: gloo, each rank a stub tracker state whose
    cost depends on the rank, the same per-frame exchange, barrier + max-over-ranks
    timing, one JSON line from rank 0."""
    import torch
    import torch.distributed as dist
    from hpe.dist import exchange_best
    if world > 1:
        dist.init_process_group("gloo")
    state = torch.zeros(27, dtype=torch.float64)
    gathered = torch.zeros(world * 27, dtype=torch.float64)

    def step(f):
        state[:26] = float(rank)
        state[26] = 10.0 + ((rank * 7 + f) % world)  # the winner changes from frame to frame
        if world > 1:
            exchange_best(state, gathered)

    for f in range(args.warmup):
        step(f)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for f in range(args.warmup, args.warmup + args.steps):
        step(f)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ranks = None
    if world > 1:  # stub ranks: the host CPU each, told apart by rank
        el, ranks = rank_report(args, world, rank, el, state.numpy(), "cpu",
                                {"pci": "cpu", "uuid": f"stub-rank{rank}", "name": "stub",
                                 "local_rank": rank})
    if rank == 0:
        print(json.dumps({"metric": "stub exchange", "value": args.steps * world / el,
                          "unit": "frames/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "stub": True, "ranks": ranks,
                          "winner_rank": int(state[0]), "winner_cost": float(state[26])}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# ------------------------------------------------------------------------- main
def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch(args)  # before anything here touches the GPU
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.stub:
        stub_main(args, world, rank)
        return 0
    import numpy as np
    import torch
    import torch.distributed as dist
    import hpe
    from hpe import synth
    from hpe.dist import GenerationExchange, exchange_best, library_exchange, subswarm_seed

    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

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
        poses = synth.trajectory(n_frames, args.seed, revert=TRAJ_REVERT)
        raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
    sizes = [len(hpe.preprocess_depth(d, True, ds)["cloud"]) for d in raw]
    if args.resident:  # frames preprocessed and resident in HBM before the timed region
        for f in range(n_frames):
            ctx.prepare_frame(f, raw[f], True, ds)
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
    gathered_host = torch.zeros(world * 27, dtype=torch.float64)
    refine = 0 if args.no_refine else 1
    gx = (GenerationExchange(ctx, args.exchange_every, args.backend)
          if args.exchange_every else None)
    # the library's own per-frame exchange: every rank joins one RCCL communicator in libhpe.so
    sub_info = library_exchange(ctx) if args.lib_exchange else None

    def step(f, ex=None):
        """One tracked frame; ex (diagnostic pass): gets the exchange's time in us."""
        if args.resident:
            ctx.select_frame(f)
            ctx.check(lib.hpe_track_frame_dev(ctx.h, P, refine, C.c_void_p(state.data_ptr())))
        else:  # frame f tracked while frame f+1 is prepared inside its refine launch
            ctx.track_pipelined(P, refine, state.data_ptr(), raw[f + 1] if f + 1 < n_frames else None)
        if args.lib_exchange:
            pass  # the library exchanged after the frame's final kernel, on its stream
        elif world > 1 and args.backend == "nccl":
            # best-of-N exchange on the tracker's own stream (no host sync)
            with torch.cuda.stream(ext):
                if ex is not None:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(ext)
                exchange_best(state, gathered, ctx=ctx)  # all-gather + hpe_pick_best
                if ex is not None:
                    e1.record(ext)
                    ex.append((e0, e1))
        elif world > 1:  # gloo: through host memory (rehearsal mode, synchronous)
            ctx.check(lib.hpe_sync(ctx.h))
            h0 = time.perf_counter()
            hs = state.cpu()
            exchange_best(hs, gathered_host)
            state.copy_(hs)
            if ex is not None:
                ex.append((time.perf_counter() - h0) * 1e6)

    dumped = []

    def dump_state():
        if args.dump:  # test mode (see --dump): one synchronisation per frame
            ctx.check(lib.hpe_sync(ctx.h))
            torch.cuda.synchronize()
            dumped.append(state.cpu().numpy().copy())

    if args.dump:
        os.makedirs(args.dump, exist_ok=True)
        if rank == 0:
            np.save(os.path.join(args.dump, "raw0.npy"), raw[0])
            np.save(os.path.join(args.dump, "x0.npy"), state[:26].cpu().numpy())
    K = args.frames_per_graph

    d_raw = None
    if K and not args.resident:  # the raw frames resident in HBM before the timed region
        d_raw = torch.from_numpy(np.ascontiguousarray(np.stack(raw), dtype=np.float32)).to(
            f"cuda:{local}")
        torch.cuda.synchronize()

    def run_sequence(first, n):  # frames first .. first+n-1, K per graph launch
        if args.resident:  # prepared frames (offline sequence API)
            ctx.track_sequence(P, refine, state.data_ptr(), first, n, K)
        else:  # raw frames, each next one prepared inside the previous frame's refine launch
            ctx.track_raw_sequence(P, refine, state.data_ptr(),
                                   d_raw.data_ptr() + first * d_raw[0].numel() * 4, n, True, ds,
                                   frames_per_graph=K)

    if not args.resident and not K:
        ctx.pipeline_begin(raw[0], True, ds)
    if K:
        run_sequence(0, args.warmup)
    else:
        for f in range(args.warmup):
            step(f)
            dump_state()
    ctx.check(lib.hpe_sync(ctx.h))
    torch.cuda.synchronize()
    state0 = state.clone()  # the diagnostic passes below restart from here: same frames, same work
    cold_ms = None
    if K:  # capture the timed range's chunk graphs once (as the per-frame graph is in warmup)
        tc = time.perf_counter()
        run_sequence(args.warmup, args.steps)
        ctx.check(lib.hpe_sync(ctx.h))
        cold_ms = (time.perf_counter() - tc) / args.steps * 1e3
        state.copy_(state0)
        torch.cuda.synchronize()
    # timed region: graph-replayed frames, nothing else on the tracker stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_s = 0.0
    if K:
        h0 = time.perf_counter()
        run_sequence(args.warmup, args.steps)
        host_s += time.perf_counter() - h0
    for f in range(args.warmup, n_frames if not K else 0):
        h0 = time.perf_counter()
        step(f)
        host_s += time.perf_counter() - h0
        dump_state()
    ctx.check(lib.hpe_sync(ctx.h))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ranks = None
    final = state.cpu().numpy()
    if world > 1:
        dev = f"cuda:{local}" if args.backend == "nccl" else "cpu"
        el, ranks = rank_report(args, world, rank, el, final, dev, device_identity(local))
    if args.dump:
        np.save(os.path.join(args.dump, f"states_rank{rank}.npy"), np.array(dumped))
    if sub_info is not None:  # in_graphs: the exchange ran inside the captured frame graphs
        sub_info.update(ctx.subswarm_info())
    # per-frame device time: the same frames again with one event pair per frame on the
    # tracker stream (not in the timed region: each timing event adds a marker, ~5 us)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    state.copy_(state0)
    torch.cuda.synchronize()
    if not args.resident and not K:
        ctx.pipeline_begin(raw[args.warmup], True, ds)
    if K:  # one event pair around the whole sequence
        ev[0][0].record(ext)
        run_sequence(args.warmup, args.steps)
        ev[0][1].record(ext)
    ex = []  # the per-frame exchange (N > 1): event pairs around it on the tracker stream
    for k, f in enumerate(range(args.warmup, n_frames if not K else 0)):
        ev[k][0].record(ext)
        step(f, ex if world > 1 else None)
        ev[k][1].record(ext)
    ctx.check(lib.hpe_sync(ctx.h))
    torch.cuda.synchronize()
    frame_us = ([a.elapsed_time(b) * 1e3 for a, b in ev] if not K else
                [ev[0][0].elapsed_time(ev[0][1]) * 1e3 / args.steps])
    ex_us = [x if isinstance(x, float) else x[0].elapsed_time(x[1]) * 1e3 for x in ex]
    if ranks is not None and ex_us:
        ranks["exchange_us"] = {
            "mean": float(np.mean(ex_us)), "median": float(np.median(ex_us)),
            "max": float(np.max(ex_us)), "frames": len(ex_us),
            "note": ("rank 0: events around the all-gather + pick on the tracker stream (the "
                     "wait for the other ranks included), second pass" if args.backend == "nccl"
                     else "rank 0: host wall time of the gloo exchange, second pass")}
    # per-kernel durations: the same frames once more with every dispatch bracketed by
    # hipExtLaunchKernel start/stop events on the tracker stream the kernels run on
    # (direct launches; kernels are identical)
    ctx.check(lib.hpe_profile_enable(ctx.h, 1))
    rev = C.c_uint64(0)
    ctx.check(lib.hpe_refine_eval_count(ctx.h, C.byref(rev), 1))  # reset
    state.copy_(state0)
    torch.cuda.synchronize()
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
    ctx.check(lib.hpe_refine_eval_count(ctx.h, C.byref(rev), 1))
    prof = {}
    for name, kid in (("k_pso_gen", 0), ("k_refine", 1), ("k_pso_init", 2), ("k_pso_final", 3),
                      ("k_preprocess", 4), ("exchange", hpe._lib.PROF_EXCHANGE)):
        nl = C.c_int32(0); tot = C.c_double(0); mn = C.c_double(0); mx = C.c_double(0)
        ctx.check(lib.hpe_profile_read_kernel(ctx.h, kid, C.byref(nl), C.byref(tot),
                                              C.byref(mn), C.byref(mx)))
        prof[name] = {"launches": nl.value, "avg_us": tot.value / max(nl.value, 1) * 1e3,
                      "min_us": mn.value * 1e3, "max_us": mx.value * 1e3,
                      "total_ms": tot.value}
    ctx.check(lib.hpe_profile_enable(ctx.h, 0))
    if args.lib_exchange:  # event pairs around the library's all-gather + pick, per frame
        xs = {"mean": prof["exchange"]["avg_us"], "min": prof["exchange"]["min_us"],
              "max": prof["exchange"]["max_us"], "frames": prof["exchange"]["launches"],
              "note": ("rank 0: hipEvents around the library's RCCL all-gather + k_pick_best on "
                       "the tracker stream (the wait for the other ranks included), in the "
                       "direct-launch profiling pass; inside the timed graphs the same nodes run "
                       "without the events")}
        if ranks is not None:
            ranks["exchange_us"] = xs
        sub_info["exchange_us"] = xs
    extra = extra_passes(args, ctx, lib, state, state0, raw, n_frames, P, refine, ds, world, rank,
                         local)
    prof["frame_graph"] = {"launches": len(frame_us), "avg_us": sum(frame_us) / len(frame_us),
                           "min_us": min(frame_us), "max_us": max(frame_us),
                           "median_us": float(np.median(frame_us)),
                           "per_frame_us": [round(x, 1) for x in frame_us],
                           "note": ("one event pair per frame, a second pass over the frames"
                                    if not K else "one event pair around the whole sequence "
                                    "(a second pass), per frame")}
    lib_path = hpe._lib.load()._name

    if rank == 0:
        n_pts = sizes[args.warmup]
        evals = P * (G + 1) * args.steps * world
        gen = roofline_entry("k_pso_gen", prof, P, n_pts, lib_path, P)
        ref_launches = prof["k_refine"]["launches"]
        ref = (roofline_entry("k_refine", prof, rev.value / ref_launches, n_pts, lib_path, P)
               if ref_launches and rev.value else None)
        kernels_rf = {"k_pso_gen": gen, "k_refine": ref}
        # the dominant kernel: the most device time per frame (hipExtLaunchKernel events)
        dom = max((k for k in kernels_rf if kernels_rf[k]),
                  key=lambda k: prof[k]["total_ms"], default=None)
        roof = dict(kernels_rf[dom]) if dom else {}
        if roof:
            roof["note"] = (
                "dominant kernel by device time per frame; algorithmic bytes per launch = "
                "evaluations per launch x (12N + 600) (SURVEY.md §8 d2), per-launch time from "
                "hipExtLaunchKernel events on the tracker stream; " + (
                    "k_pso_gen = one generation of the swarm per launch, one particle per "
                    "workgroup" if dom == "k_pso_gen" else
                    "k_refine = refine_init_pose as ONE workgroup (a serial chain of "
                    "evaluations), plus the next frame's preparation workgroups") +
                "; latency-bound (dependent generations / a serial line search), DESIGN.md §5")
            roof["limiter"] = "latency"
        dominant = {"kernel": dom,
                    "ms_per_frame": {k: prof[k]["total_ms"] / max(args.steps, 1)
                                     for k in ("k_pso_gen", "k_refine", "k_pso_init",
                                               "k_pso_final")}}
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
            "vs_baseline": None,  # set below from the same-run CPU baseline
            "dtype": "f32+f64",
            "data": (f"recorded: {n_frames} *_depth.bin frames from {args.frames}" if args.frames
                     else "synthetic: seeded 26-DOF trajectory rendered from the 48-sphere "
                          "model into 240x320 float32 mm depth (no MSRA Subject1 on the box)"),
            "config": {"workload": (f"{args.config} = {CONFIGS[args.config][2]}; step = one "
                                    "tracked frame = " + ("" if args.resident else
                                    "next_frame preprocessing (GPU, fused into the refine "
                                    "launch) + ") + "refine_init_pose + pso_evolve + "
                                    "cal_cost(bestp)" + (
                                        f"; prepared frames resident in HBM, tracked by the "
                                        f"offline sequence API, {K} frames per graph launch"
                                        if K and args.resident else
                                        f"; raw float32 mm depth frames resident in HBM, "
                                        f"hpe_track_raw_sequence_dev, {K} frames per graph "
                                        f"launch" if K else
                                        "" if args.resident else
                                        "; raw frames from host memory (zero-copy over "
                                        "PCIe), one hpe_track_pipelined graph per frame")),
                       "frames_per_graph": K or 1,
                       "particles": P, "generations": G, "maxiter": G + 1,
                       "trajectory": (None if args.frames else
                                      {"seed": args.seed, "revert": TRAJ_REVERT,
                                       "frames": n_frames}),
                       "cloud_points": n_pts, "refine": bool(refine),
                       "refine_form": extra["refine_form"],
                       "refine_kernel": extra["refine_kernel"],
                       "exchange_form": (
                           "library: libhpe.so's RCCL all-gather + pick after every frame, "
                           + ("captured in the frame graphs" if sub_info["in_graphs"] else
                              "direct launches (the capture fell back)")
                           + f" (hpe_subswarm_init), {sub_info['nranks']} rank(s)"
                           if args.lib_exchange else
                           "torch: torch.distributed all_gather_into_tensor + hpe_pick_best per "
                           f"frame on the tracker stream ({args.backend})" if world > 1 else
                           "none (one GPU)"),
                       "exchange": ("once per frame (best of N subswarms)" if not args.exchange_every
                                    else f"every {args.exchange_every} generations + per frame "
                                         "(ICP-PSO style, non-reference)"),
                       "parallelism": f"subswarms x{world}, all-gather best per frame"
                                      + ("" if world == 1 else f" ({args.backend}"
                                         + (", ranks sharing cuda:0)" if args.same_device
                                            else ")"))},
            "tracked_fps": args.steps / el,
            "final_cost": float(final[26]),
            "tracking_err_mm": ({"sum_wrist_tips_mean": float(np.mean(errs)),
                                 "per_joint_mean": float(np.mean(errs) / 6),
                                 "note": "gnd_truth_err (costfunc.cpp:476-507) vs the synthetic "
                                         "trajectory's true poses, second pass over the frames"}
                                if errs else None),
            "roofline": roof or None,
            "dominant_kernel": dominant,
            "roofline_kernels": kernels_rf,
            "refine_exact_ms_per_step": extra["refine_exact_ms_per_step"],
            "per_frame_graph_ms_per_step": extra["per_frame_graph_ms_per_step"],
            "scaling_baseline_ms_per_step": extra["scaling_baseline_ms_per_step"],
            "exchange_off_ms_per_step": extra["exchange_off_ms_per_step"],
            "subswarm": sub_info,
            "extra_passes_note": extra["note"],
            "refine_evals_per_frame": rev.value / max(ref_launches, 1),
            "kernels": prof,
            "host_us_per_step": host_s / args.steps * 1e6,
            "cold_graphs_ms_per_step": cold_ms,
            "ranks": ranks,
            "lib_sha256": lib_sha256(lib_path),
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args, raw if args.frames else None)
            line["cpu_baseline"] = cb
            line["speedup_vs_cpu"] = {"particle_evals": line["value"] / cb["value"],
                                      "tracked_fps": line["tracked_fps"] / cb["tracked_fps"]}
            # nothing is published for this metric, so vs_baseline stays
            # null; the ratio to the same-run CPU restatement is
            # speedup_vs_cpu
            line["vs_baseline_basis"] = ("null: BASELINE.md publishes no number for this "
                                         "metric; see speedup_vs_cpu for the same-run CPU "
                                         "baseline")
        print(json.dumps(line), flush=True)
    if gx is not None:
        if gx.error is not None:
            raise SystemExit(f"rank {rank}: generation exchange failed: {gx.error!r}")
        gx.close()
    hand.ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    # a normal interpreter exit: rocprofv3 writes its traces from exit handlers
    sys.exit(main() or 0)
