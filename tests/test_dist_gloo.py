"""Multi-rank path on the CPU (gloo, world_size 2 and 8): the per-frame best-of-subswarms
exchange of hpe.dist (the code bench.py runs over RCCL), with the subswarms computed by
the C oracle so the expected winner is known independently.  SURVEY.md §8e."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import hand_data
import oracle_np


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _subswarm(rank, frames_seed=31, P=8, maxiter=3):
    import oracle_c
    from hpe.dist import subswarm_seed
    o = oracle_c.load(build=False)
    geo, rad = hand_data.geometry_cm()
    h = o.hand(geo, rad)
    nh = oracle_np.Hand(geo, rad)
    poses = hand_data.trajectory(2, seed=frames_seed)
    obs = o.preprocess(oracle_np.render_depth_mm(nh, poses[1]))
    ub, lb, sd = oracle_np.reference_bounds()
    bp, bc, _ = o.pso_evolve(h, obs, poses[0], P, maxiter, lb, ub, sd, seed=subswarm_seed(rank),
                             nthreads=1)
    return np.concatenate([bp, [bc]])


def _worker(rank, world, port, out_dir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hpe.dist import exchange_best
    if mode == "pso":
        st = torch.from_numpy(_subswarm(rank))
    elif mode == "tie":
        st = torch.full((27,), float(rank), dtype=torch.float64)
        st[26] = 5.0
    elif mode == "libid":
        # hpe.dist.library_exchange's set-up on gloo ranks with a stand-in context: rank 0's
        # unique id reaches every rank, and every rank joins with (world, its rank)
        import hpe
        import hpe.dist as hd

        class Ctx:
            device = 0

            def subswarm_init(self, uid, nranks, rank):
                self.args = (uid, nranks, rank)

            def subswarm_info(self):
                return {"nranks": self.args[1], "rank": self.args[2]}

        uid = bytes((7 * k + 3) % 256 for k in range(128))
        hpe.subswarm_unique_id = lambda: uid if rank == 0 else bytes(128)  # rank 0 draws
        ctx = Ctx()
        info = hd.library_exchange(ctx)
        st = torch.tensor(list(ctx.args[0]) + [ctx.args[1], ctx.args[2], info["nranks"]],
                          dtype=torch.float64)
    else:  # nan: rank 0 diverged
        st = torch.full((27,), float(rank), dtype=torch.float64)
        st[26] = float("nan") if rank == 0 else 7.0
    if mode != "libid":
        exchange_best(st)
    np.save(os.path.join(out_dir, f"r{rank}.npy"), st.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, mode, world=2):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world,
                       join=True, start_method="spawn")
    return [np.load(tmp_path / f"r{r}.npy") for r in range(world)]


def test_exchange_picks_best_subswarm(tmp_path):
    res = _run(tmp_path, "pso")
    expect = [_subswarm(r) for r in range(2)]
    win = int(np.argmin([e[26] for e in expect]))
    for r in res:
        np.testing.assert_array_equal(r, expect[win])
    assert expect[0][26] != expect[1][26]  # distinct streams per rank


def test_exchange_eight_ranks(tmp_path):
    """The 8-GPU shape of config 5 (one subswarm per rank, seeds 1000..1007) on 8 gloo
    ranks: every rank ends with the oracle's best of the eight subswarms."""
    res = _run(tmp_path, "pso", world=8)
    expect = [_subswarm(r) for r in range(8)]
    win = int(np.argmin([e[26] for e in expect]))
    for r in res:
        np.testing.assert_array_equal(r, expect[win])
    assert len({e[26] for e in expect}) == 8


def test_exchange_tie_lowest_rank(tmp_path):
    for r in _run(tmp_path, "tie"):
        assert r[0] == 0.0 and r[26] == 5.0


def test_exchange_nan_never_wins(tmp_path):
    for r in _run(tmp_path, "nan"):
        assert r[0] == 1.0 and r[26] == 7.0


def test_single_rank_is_identity():
    from hpe.dist import pick_best, subswarm_seed
    assert subswarm_seed(0) == 1000
    g = torch.tensor([[1.0] * 26 + [3.0], [2.0] * 26 + [3.0]], dtype=torch.float64)
    assert pick_best(g)[0] == 1.0


def test_library_exchange_setup_broadcasts_rank0_id(tmp_path):
    """hpe.dist.library_exchange (bench.py's N > 1 set-up of the library's own RCCL
    communicator, hpe_subswarm_init): on 2 gloo ranks every rank receives rank 0's 128-byte
    unique id through the process group and joins as (world 2, its own rank)."""
    res = _run(tmp_path, "libid")
    uid = [(7 * k + 3) % 256 for k in range(128)]
    for r, st in enumerate(res):
        assert list(st[:128].astype(int)) == uid
        assert st[128] == 2 and st[129] == r and st[130] == 2
