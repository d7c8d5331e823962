"""Several camera streams tracked concurrently on one GPU (serving form of test_full's loop,
testmodel.cpp:117-139): S independent contexts (hpe_ctx: own buffers, own HIP stream, own
graphs), each running the pipelined tracker on its own synthetic sequence; the host
enqueues their frames round-robin, so the single-workgroup refine of one stream overlaps
the swarm generations of the others.

Checks that every stream's per-frame {bestp, cost} in the concurrent run is bit-identical
to the same stream tracked alone, then prints one JSON line per stream count with the
aggregate tracked FPS.  Usage (GPU box): python tools/serve_streams.py [--streams 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "hand-pose-estimation_amd")]

import numpy as np  # noqa: E402


def make_streams(S, n_frames, P=256, G=30, seed0=0):
    import torch
    import hpe
    from hpe import synth
    streams = []
    ub, lb, sd = hpe.reference_bounds()
    for s in range(S):
        hand = hpe.reference_hand(device=0)
        ctx = hand.ctx
        poses = synth.trajectory(n_frames, seed0 + s, revert=0.02)
        raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
        pso = hpe.PSO()
        pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, G + 1, 1e-8, 1e-8)
        pso._push(ctx)
        state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
        streams.append(dict(hand=hand, ctx=ctx, raw=raw, x0=poses[0], state=state, P=P))
    return streams


def run(streams, frames, record=False):
    """Track frames[0] .. frames[-1] of every stream, round-robin; returns per-stream
    per-frame states when record (one host sync per frame: not for timing)."""
    import torch
    for st in streams:
        st["state"].zero_()
        st["state"][:26] = torch.from_numpy(np.asarray(st["x0"], dtype=np.float64))
        st["hist"] = []
    torch.cuda.synchronize()
    for st in streams:
        st["ctx"].pipeline_begin(st["raw"][frames[0]], True, True)
    for f in frames:
        for st in streams:
            nxt = st["raw"][f + 1] if f + 1 <= frames[-1] else None
            st["ctx"].track_pipelined(st["P"], 1, st["state"].data_ptr(), nxt)
        if record:
            for st in streams:
                st["ctx"].check(st["ctx"].lib.hpe_sync(st["ctx"].h))
                st["hist"].append(st["state"].cpu().numpy().copy())
    for st in streams:
        st["ctx"].check(st["ctx"].lib.hpe_sync(st["ctx"].h))
    torch.cuda.synchronize()
    return [np.array(st["hist"]) for st in streams] if record else None


def check_against_alone(streams, frames):
    """Concurrent per-frame states == each stream tracked alone (bit for bit)."""
    together = run(streams, frames, record=True)
    for s, st in enumerate(streams):
        alone = run([st], frames, record=True)[0]
        if not np.array_equal(alone, together[s]):
            d = np.abs(alone - together[s]).max()
            raise AssertionError(f"stream {s}: concurrent run differs from alone (max {d})")
    return together


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import torch
    torch.cuda.is_available()
    counts = [int(x) for x in a.streams.split(",")]
    n = a.warmup + a.steps
    allst = make_streams(max(counts), n)
    check_against_alone(allst[:min(3, max(counts))], list(range(6)))
    for S in counts:
        sts = allst[:S]
        run(sts, list(range(a.warmup)))  # graphs captured
        t0 = time.perf_counter()
        run(sts, list(range(a.warmup, n)))
        el = time.perf_counter() - t0
        fps = S * a.steps / el
        print(json.dumps({"streams": S, "frames_per_stream": a.steps,
                          "aggregate_tracked_fps": fps,
                          "aggregate_particle_evals_per_s": fps * 256 * 31,
                          "ms_per_round": el / a.steps * 1e3,
                          "workload": "256 p x 30 gen, refine on, N = 250, pipelined raw depth "
                                      "in, one context per stream, seeds 0..S-1"}), flush=True)
    for st in allst:
        st["ctx"].close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
