"""Multi-GPU layout of the env batch: one process per GPU, contiguous env
shards, no collective on the data path (weak scaling).

The reference shards the same way under pmap (ippo_rnn_JAXMARL_pmap.py:292-332:
env state reshaped to (N_DEVICES, NUM_ENVS / N_DEVICES, ...), env params
replicated).  The only collectives here are for timing: a barrier and the
max over ranks of the elapsed time.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional, Tuple


@dataclass
class Ranks:
    world: int
    rank: int
    local: int
    dist: Optional[object]  # torch.distributed when world > 1


def init_from_env(backend: str = "nccl") -> Ranks:
    """Read torchrun's WORLD_SIZE / RANK / LOCAL_RANK; init the process group when world > 1.

    backend "nccl" is RCCL on ROCm (one GPU per process); "gloo" runs on CPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    d = None
    if world > 1:
        import torch
        import torch.distributed as d
        if backend == "nccl":
            torch.cuda.set_device(local)
            d.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            d.init_process_group(backend)
    return Ranks(world, rank, local, d)


def env_slice(rank: int, envs_per_rank: int) -> Tuple[int, int]:
    """Global env indices [start, stop) owned by `rank` (contiguous blocks)."""
    return rank * envs_per_rank, (rank + 1) * envs_per_rank


def rank_keys(all_keys, rank: int, envs_per_rank: int):
    """This rank's env keys from the global split `all_keys` = split(master, world*E + 1);
    row 0 is the master carry (Speed_test.py:142-147), envs start at row 1."""
    a, b = env_slice(rank, envs_per_rank)
    return all_keys[1 + a:1 + b]


def barrier(r: Ranks) -> None:
    if r.dist is not None:
        r.dist.barrier()


def max_over_ranks(r: Ranks, x: float, device=None) -> float:
    """max of a per-rank scalar (the timing reduction of bench.py)."""
    if r.dist is None:
        return float(x)
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    r.dist.all_reduce(t, op=r.dist.ReduceOp.MAX)
    return float(t.item())


def finalize(r: Ranks) -> None:
    if r.dist is not None:
        r.dist.destroy_process_group()
