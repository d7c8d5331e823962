"""Multi-GPU subswarms: one process per GPU, each running its own
complete pso_evolve (own topology, seed 1000 + rank), and ONE exchange per tracked frame:
an all-gather of the 27-double tracker state {bestp[26], cost} over RCCL (xGMI) after
which every rank adopts the lexicographic minimum (cost, rank).  RCCL has no MINLOC, hence
all-gather + argmin rather than all-reduce; 216 B per rank, latency-bound.

Because gbest never enters the reference velocity update (PSO.cpp:824-832), exchanging
once per frame is exactly "best of N independent swarms"; the winner becomes every
rank's next-frame x0 (testmodel.cpp:138).

library_exchange sets up the same per-frame exchange INSIDE libhpe.so (hpe_subswarm_init):
the library's own RCCL communicator all-gathers and picks after every tracked frame on the
tracker stream, captured into the tracking graphs with the frames -- so N ranks run exactly
the N = 1 loop (8 frames per graph launch) plus one all-gather per frame.  exchange_best is
the torch.distributed form of the same step (one graph per frame; and the gloo rehearsal).

GenerationExchange adds the opt-in ICP-PSO style exchange (NOT the reference algorithm):
every K generations each rank's best pbest is all-gathered and the best over all ranks
becomes an extra informant candidate of every particle (hpe_set_exchange).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

STATE_LEN = 27  # bestp[26] + cost
BASE_SEED = 1000  # arma_rng::set_seed(1000), PSO.cpp:722


def subswarm_seed(rank: int, base: int = BASE_SEED) -> int:
    """Rank r's PSO stream; rank 0 reproduces the single-GPU (reference-seeded) run."""
    return base + rank


def pick_best(gathered: torch.Tensor) -> torch.Tensor:
    """Row of the (world, 27) gathered states with the smallest cost; ties -> lowest
    rank (torch.argmin returns the first minimum); NaN costs never win."""
    c = torch.nan_to_num(gathered[:, STATE_LEN - 1], nan=float("inf"))
    return gathered[torch.argmin(c)]


def exchange_best(state: torch.Tensor, gathered: torch.Tensor | None = None,
                  group=None, ctx=None) -> torch.Tensor:
    """In place: state <- best state over all ranks.  Runs on the current stream (the
    caller wraps it in the tracker's stream so no host synchronisation is needed).
    ctx (a device state and the tracker context whose stream is current): the pick is
    hpe_pick_best, one launch on that stream, instead of pick_best's torch kernels."""
    world = dist.get_world_size(group)
    if world == 1:
        return state
    if gathered is None:
        gathered = state.new_empty(world * STATE_LEN)
    dist.all_gather_into_tensor(gathered, state, group=group)
    if ctx is not None and state.is_cuda:
        import ctypes as C
        ctx.check(ctx.lib.hpe_pick_best(ctx.h, C.c_void_p(gathered.data_ptr()), world,
                                        C.c_void_p(state.data_ptr())))
    else:
        state.copy_(pick_best(gathered.view(world, STATE_LEN)))
    return state


def library_exchange(ctx, group=None) -> dict:
    """Every rank of `group` (default: the world; world 1 without a process group) joins one
    RCCL communicator owned by ctx's library: rank 0 draws the unique id, the process group
    broadcasts it (a CUDA tensor on "nccl", a CPU one on "gloo"), then hpe_subswarm_init on
    every rank (collective).  Returns ctx.subswarm_info()."""
    from . import subswarm_unique_id
    if dist.is_initialized():
        world, rank = dist.get_world_size(group), dist.get_rank(group)
    else:
        world, rank = 1, 0
    uid = subswarm_unique_id() if rank == 0 else bytes(128)
    if world > 1:
        dev = (torch.device("cuda", ctx.device) if dist.get_backend(group) == "nccl"
               else torch.device("cpu"))
        t = torch.tensor(list(uid), dtype=torch.uint8, device=dev)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(t, src=src, group=group)
        uid = bytes(t.cpu().tolist())
    ctx.subswarm_init(uid, world, rank)
    return ctx.subswarm_info()


class GenerationExchange:
    """The opt-in per-generation exchange (hpe_set_exchange; ICP-PSO style, labelled
    non-reference: the reference's gbest never enters the velocity, PSO.cpp:824-832).

    After every `every`-th generation the library writes this rank's best pbest
    {pose, cost} into `ext` (27 doubles on the context's device) and calls back here; the
    callback replaces it by the best over all ranks (exchange_best: all-gather + lowest
    cost, ties to the lowest rank) ON THE CONTEXT'S STREAM, so the next generation reads it
    without a host synchronisation (nccl = RCCL).  backend "gloo" (a rehearsal: several
    ranks on one GPU) goes through host memory and synchronises the stream.  Keep the
    object alive while the context tracks; close() turns the exchange off."""

    def __init__(self, ctx, every: int, backend: str = "nccl", group=None):
        import ctypes as C

        from . import _lib
        self.ctx, self.every, self.backend, self.group = ctx, every, backend, group
        dev = torch.device("cuda", ctx.device)
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.ext = torch.zeros(STATE_LEN, dtype=torch.float64, device=dev)
        self.gathered = torch.zeros(world * STATE_LEN, dtype=torch.float64,
                                    device=dev if backend == "nccl" else "cpu")
        self.stream = torch.cuda.ExternalStream(ctx.lib.hpe_stream(ctx.h), device=dev)
        self.calls = 0
        self.error = None
        self._cb = _lib.EXCHANGE_FN(self._call)  # referenced for the context's lifetime
        ctx.check(ctx.lib.hpe_set_exchange(ctx.h, every, C.c_void_p(self.ext.data_ptr()),
                                           C.cast(self._cb, C.c_void_p), None))

    def _call(self, user, d_ext, generation):
        try:
            if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
                pass  # one swarm: its own best is the candidate
            elif self.backend == "nccl":
                with torch.cuda.stream(self.stream):
                    exchange_best(self.ext, self.gathered, self.group)
            else:
                self.stream.synchronize()
                h = self.ext.cpu()
                exchange_best(h, self.gathered, self.group)
                with torch.cuda.stream(self.stream):
                    self.ext.copy_(h)
            self.calls += 1
            return 0
        except Exception as e:  # noqa: BLE001 -- reported through the C ABI's status
            self.error = e
            return 1

    def close(self):
        if self.ctx is not None and self.ctx.h:
            self.ctx.check(self.ctx.lib.hpe_set_exchange(self.ctx.h, 0, None, None, None))
        self.ctx = None
