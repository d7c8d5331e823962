"""Reference hand geometry (misc/hgeo.dat, misc/rad.dat values, committed as package
data) and synthetic frame helpers shared by the tests."""
import json
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
HAND_JSON = ROOT / "hand-pose-estimation_amd" / "hpe" / "hand_subject1.json"


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
