"""Compare a tools/seq_dump.py dump with the C oracle frame by frame (oracle started from
the GPU's previous pose: per-frame parity) and report the worst frames.
usage: seq_compare.py DUMP.npz [first] [last]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "tests")]
import hand_data  # noqa: E402
import oracle_c  # noqa: E402
import oracle_np  # noqa: E402

d = np.load(sys.argv[1])
o = oracle_c.load()
geo, rad = hand_data.geometry_cm()
h = o.hand(geo, rad)
ub, lb, sd = oracle_np.reference_bounds()
P, maxiter = int(d["P"]), int(d["maxiter"])
raw, gx, gc, poses, ev = d["raw"], d["gx"], d["gc"], d["poses"], d["evals"]
a = int(sys.argv[2]) if len(sys.argv) > 2 else 0
b = int(sys.argv[3]) if len(sys.argv) > 3 else len(gx)
rows = []
for f in range(a, b):
    obs = o.preprocess(raw[f])
    x0 = poses[0] if f == 0 else gx[f - 1]
    xr, er = o.refine(h, obs, x0)
    xp, cp, tr = o.pso_evolve(h, obs, xr, P, maxiter, lb, ub, sd, seed=1000)
    cr = o.cal_cost(h, obs, xp)
    dp = np.abs(gx[f] - xp).max()
    dc = abs(gc[f] - cr) / abs(cr) if np.isfinite(cr) else (0.0 if np.isnan(gc[f]) else np.inf)
    rows.append((f, dp, dc, ev[f], er))
    if dp > 1e-6 or dc > 1e-8 or ev[f] != er:
        print(f"frame {f}: |dpose| {dp:.3g}  dcost {dc:.3g}  refine evals gpu {ev[f]} oracle {er}")
r = np.array(rows)
print(f"frames {a}..{b - 1}: max |dpose| {r[:, 1].max():.3g} (frame {int(r[r[:, 1].argmax(), 0])}), "
      f"max dcost {r[:, 2].max():.3g}, refine eval mismatches {(r[:, 3] != r[:, 4]).sum()}")

# free-running oracle over the same frames: how far the two trajectories drift apart
x = poses[0].copy()
drift = []
for f in range(len(gx)):
    obs = o.preprocess(raw[f])
    x, _ = o.refine(h, obs, x)
    x, _, _ = o.pso_evolve(h, obs, x, P, maxiter, lb, ub, sd, seed=1000)
    drift.append(np.abs(x - gx[f]).max())
drift = np.array(drift)
for t in (1e-9, 1e-8, 1e-7, 1e-6, 1e-5, 1e-3, 1e-1):
    k = np.nonzero(drift > t)[0]
    print(f"free-running: first frame with |dpose| > {t:g}: {k[0] if len(k) else None}")
print("free-running max |dpose|", drift.max(), "median", np.median(drift))
