"""The multi-workgroup refine's failure mode (clouds > 2048 points, hpe_kernels.hip
mw_helper / mw_collect): every hand-off wait is bounded, and a wait that runs out must
leave that frame visibly failed -- its pose and cost NaN in the device state, which never
wins an exchange -- and make the NEXT tracking call return an error, without a host
synchronisation per frame (the flag is mirrored into pinned host memory).

HPE_MW_SPIN=0 (read at hpe_create) gives every wait a budget of zero polls, so the first
hand-off of every launch times out deterministically.  A default context on the same
frames succeeds (the budget is the only difference)."""
import numpy as np
import pytest

import hand_data
import oracle_np

pytestmark = pytest.mark.gpu


def _run(gh, raw, P=32, maxiter=6):
    import torch
    import hpe
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    pso._push(gh.ctx)
    state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    state[:26] = torch.from_numpy(hand_data.trajectory(1)[0])
    torch.cuda.synchronize()
    gh.ctx.pipeline_begin(raw[0], True, False)  # full cloud: the multi-workgroup refine
    gh.ctx.track_pipelined(P, 1, state.data_ptr(), raw[1])
    torch.cuda.synchronize()  # the frame has run (no hpe_sync: the flag is not consumed)
    return state


def test_mw_refine_timeout_is_visible(monkeypatch):
    import hpe
    poses = hand_data.trajectory(3, seed=8, revert=0.02)
    monkeypatch.setenv("HPE_MW_SPIN", "0")
    gh = hpe.reference_hand(device=0)
    raw = [np.ascontiguousarray(gh.ctx.render_depth(th)) for th in poses]
    assert len(hpe.preprocess_depth(raw[0], True, False)["cloud"]) > 2048
    state = _run(gh, raw)
    s = state.cpu().numpy()
    assert np.isnan(s[26]), s  # the failed frame's cost
    with pytest.raises(hpe.HpeError, match="timed out"):  # the next call reports it
        gh.ctx.track_pipelined(32, 1, state.data_ptr(), raw[2])
    assert gh.ctx.lib.hpe_sync(gh.ctx.h) == 0  # reported once, then cleared
    gh.ctx.frame_token = None
    gh.ctx.close()
    monkeypatch.delenv("HPE_MW_SPIN")
    ok = hpe.reference_hand(device=0)  # default budget, same frames
    s = _run(ok, raw).cpu().numpy()
    assert np.isfinite(s).all()
    assert ok.ctx.lib.hpe_sync(ok.ctx.h) == 0
    ok.ctx.frame_token = None
