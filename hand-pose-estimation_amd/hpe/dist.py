"""Multi-GPU subswarms: one process per GPU, each running its own
complete pso_evolve (own topology, seed 1000 + rank), and ONE exchange per tracked frame:
an all-gather of the 27-double tracker state {bestp[26], cost} over RCCL (xGMI) after
which every rank adopts the lexicographic minimum (cost, rank).  RCCL has no MINLOC, hence
all-gather + argmin rather than all-reduce; 216 B per rank, latency-bound.

Because gbest never enters the reference velocity update (PSO.cpp:824-832), exchanging
once per frame is exactly "best of N independent swarms"; the winner becomes every
rank's next-frame x0 (testmodel.cpp:138).
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
                  group=None) -> torch.Tensor:
    """In place: state <- best state over all ranks.  Runs on the current stream (the
    caller wraps it in the tracker's stream so no host synchronisation is needed)."""
    world = dist.get_world_size(group)
    if world == 1:
        return state
    if gathered is None:
        gathered = state.new_empty(world * STATE_LEN)
    dist.all_gather_into_tensor(gathered, state, group=group)
    state.copy_(pick_best(gathered.view(world, STATE_LEN)))
    return state
