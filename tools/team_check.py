"""Diagnostic (GPU): refine_init_pose in the three forms of the hand-frame refine --
k_refine (HPE_REFINE_TEAM=0), the team kernel's leader alone (solo) and leader + helpers
(team) -- on the bench trajectory's frames: results and evaluation counts must be
bit-identical across the forms and repeat runs, and equal the oracle's mirror (or a near-tie
replay of it).  Then the tracked-frame time of each form (256 x 30, refine on, raw frames
resident, 8 per graph).

Usage: python tools/team_check.py [frames] [timed_frames]"""
import ctypes as C
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "hand-pose-estimation_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import torch  # noqa: E402

torch.cuda.is_available()
import hand_data  # noqa: E402
import hpe  # noqa: E402
import oracle_c  # noqa: E402
import oracle_np  # noqa: E402
from hpe import _lib, synth  # noqa: E402

NF = int(sys.argv[1]) if len(sys.argv) > 1 else 12
NT = int(sys.argv[2]) if len(sys.argv) > 2 else 40
FORMS = ("0", "solo", "1")


def make(form):
    os.environ["HPE_REFINE_TEAM"] = form
    return hpe.reference_hand(device=0)


ora = oracle_c.load(build=False)
geo, rad = hand_data.geometry_cm()
oh = ora.hand(geo, rad)
hands = {f: make(f) for f in FORMS}
ub, lb, sd = oracle_np.reference_bounds()

# the failing round-5 frame (test_config2_single_frame_256x30) and the bench sequence
cases = []
p2 = hand_data.trajectory(4, seed=2)
cases.append(("cfg2", p2[2], p2[3]))
seq = synth.trajectory(NF + 3, 0, revert=0.02)
for f in range(3, 3 + NF):
    cases.append((f"bench{f}", seq[f - 1], seq[f]))

bad = 0
for name, x0, pose in cases:
    depth = hands["0"].ctx.render_depth(pose)
    obs = ora.preprocess(depth)
    xr, er = ora.refine(oh, obs, x0, rigid=True)
    res = {}
    for form, h in hands.items():
        om = hpe.observedmodel()
        om.downsample = True
        om.set_depth_mm(depth)
        cf = hpe.costfunc(h, om)
        outs = []
        for rep in range(2):
            pso = hpe.PSO()
            x = x0.copy()
            pso.refine_init_pose(x, cf)
            outs.append((x.copy(), pso.last_refine_evals))
        same = all(np.array_equal(outs[0][0], o[0]) and outs[0][1] == o[1] for o in outs)
        res[form] = (outs[0][0], outs[0][1], same)
    x_0, e_0, _ = res["0"]
    line = f"{name:8s} oracle evals {er:4d}"
    for form in FORMS:
        x, e, same = res[form]
        ident = np.array_equal(x, x_0) and e == e_0
        line += f" | {form}: evals {e:4d} rep-same {same} ==k_refine {ident} |dx| {np.max(np.abs(x - xr)):.1e}"
        if not (same and ident):
            bad += 1
    if res["0"][1] != er:
        fl = hand_data.tie_replay(ora, oh, obs, x0, res["0"][1], True, 1e-13, pose=res["0"][0])
        line += f" tie-replay {fl}"
    print(line, flush=True)
print("MISMATCHES", bad, flush=True)

# timing: the bench loop (raw frames resident, 8 per graph) per form
raw = [np.ascontiguousarray(hands["0"].ctx.render_depth(th)) for th in synth.trajectory(NT + 4, 0, revert=0.02)]
for form, h in hands.items():
    ctx = h.ctx
    ctx.check(ctx.lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                         _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 31, 1e-8, 1e-8))
    d_raw = torch.from_numpy(np.stack(raw)).cuda()
    hist = torch.zeros((len(raw), 27), dtype=torch.float64, device="cuda:0")
    ts = []
    for rep in range(3):
        st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
        st[:26] = torch.from_numpy(synth.trajectory(1, 0, revert=0.02)[0])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.track_raw_sequence(256, 1, st.data_ptr(), d_raw.data_ptr(), len(raw), frames_per_graph=8,
                               d_hist_ptr=hist.data_ptr())
        ctx.check(ctx.lib.hpe_sync(ctx.h))
        ts.append((time.perf_counter() - t0) / len(raw) * 1e3)
    h_fin = hist.cpu().numpy()
    if form == "0":
        ref_hist = h_fin
    print(f"form {form:5s}: ms/frame {['%.4f' % v for v in ts]}  hist==k_refine {np.array_equal(h_fin, ref_hist)}",
          flush=True)
