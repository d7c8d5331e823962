"""Synthetic input for bench and smoke runs (no MSRA data exists on the GPU box).

A seeded, smooth 26-DOF pose trajectory starting at test_full's x0
(testmodel.cpp:38-40), rendered by the GPU into 240x320 float32 mm depth frames in the
reference .bin layout (observedmodel.cpp:280-308), preprocessed like next_frame
(observedmodel.cpp:420-430) and stored resident in HBM frame slots.
"""
from __future__ import annotations

import numpy as np

from . import X0, Context, preprocess_depth, reference_bounds


def trajectory(n_frames: int, seed: int = 0, step: float = 0.15,
               revert: float = 0.0) -> np.ndarray:
    """revert > 0 pulls the pose back towards x0 (long sequences stay in view)."""
    rng = np.random.default_rng(seed)
    ub, lb, sd = reference_bounds()
    poses = [X0.copy()]
    vel = np.zeros(26)
    for _ in range(n_frames - 1):
        vel = 0.8 * vel + 0.2 * rng.standard_normal(26) * sd * step
        vel += revert * (X0 - poses[-1])
        poses.append(np.clip(poses[-1] + vel, lb, ub))
    return np.array(poses)


def load_sequence(ctx: Context, n_frames: int, seed: int = 0, downsample: bool = True,
                  focal: float = 241.42, first_slot: int = 0):
    """Render + preprocess + store n_frames into slots first_slot..; returns
    (poses, cloud sizes)."""
    poses = trajectory(n_frames, seed)
    sizes = []
    for f, th in enumerate(poses):
        d = ctx.render_depth(th, focal)
        o = preprocess_depth(d, True, downsample, focal)
        ctx.store_frame(first_slot + f, o["depth_cm"], o["dt"], o["cloud"], o["scale"],
                        o["dtmax"], o["K"])
        sizes.append(len(o["cloud"]))
    return poses, sizes
