"""Reference hand geometry (misc/hgeo.dat, misc/rad.dat values, committed as package
data) and synthetic frame helpers shared by the tests."""
import json
import os
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
HAND_JSON = ROOT / "hand-pose-estimation_amd" / "hpe" / "hand_subject1.json"

# The GPU contexts' refine form (hpe_create reads HPE_REFINE_EXACT): the hand-frame refine
# by default, compared with the oracle's mirror of it; the reference's chain under
# HPE_REFINE_EXACT=1, compared with the oracle's restatement (tests/test_rigid.py bounds
# the distance between the two).
REFINE_RIGID = os.environ.get("HPE_REFINE_EXACT", "0") != "1"


def geometry_cm():
    d = json.loads(HAND_JSON.read_text())
    return np.array(d["hgeo_mm"]) / 10.0, np.array(d["rad_mm"]) / 10.0


def random_thetas(rng, P, x0=None, spread=1.0):
    import oracle_np
    x0 = oracle_np.X0 if x0 is None else x0
    ub, lb, sd = oracle_np.reference_bounds()
    th = x0[None, :] + rng.standard_normal((P, 26)) * sd[None, :] * spread
    return np.clip(th, lb, ub)


def trajectory(n_frames, seed=0, revert=0.0):
    """Smooth seeded pose sequence starting at testmodel.cpp's x0;
    revert > 0 pulls the pose back towards x0 so that long sequences stay in view."""
    import oracle_np
    rng = np.random.default_rng(seed)
    ub, lb, sd = oracle_np.reference_bounds()
    poses = [oracle_np.X0.copy()]
    vel = np.zeros(26)
    for _ in range(n_frames - 1):
        vel = 0.8 * vel + 0.2 * rng.standard_normal(26) * sd * 0.15
        vel += revert * (oracle_np.X0 - poses[-1])
        poses.append(np.clip(poses[-1] + vel, lb, ub))
    return np.array(poses)


def tie_replay(oracle, ora_hand, obs, x0, evals, rigid, tie, pose=None, depth=2):
    """Explain a refine that took `evals` evaluations where the oracle's run from x0 took
    another number: replay the oracle with near-tie decisions (relative margin < tie)
    inverted -- one, then pairs (the second chosen among the flipped run's own later
    near-ties) -- until a replay takes exactly `evals` evaluations (and, if given, reaches
    `pose` within 1e-6).  Returns [(decision, margin), ...] of the flips, or None when no
    combination of near-ties explains it (a real divergence)."""
    import numpy as np

    def run(fl):
        return oracle.refine_log(ora_hand, obs, x0, rigid=rigid, flips=fl)

    _, _, m = run(())
    frontier = [((), (), m)]
    for _ in range(depth):
        nxt = []
        for fl, ms, mm in frontier:
            start = fl[-1] + 1 if fl else 0
            for k in np.flatnonzero(mm < tie):
                if k < start:
                    continue
                f2, m2 = fl + (int(k),), ms + (float(mm[k]),)
                xf, ef, mf = run(f2)
                if ef == evals and (pose is None or np.max(np.abs(xf - pose)) < 1e-6):
                    return list(zip(f2, m2))
                nxt.append((f2, m2, mf))
        frontier = nxt
    return None
