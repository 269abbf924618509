"""Env-sharded data parallelism: one process per GPU, torch.distributed over RCCL
("nccl" backend on ROCm) -- gloo for CPU tests.

Partitioning: rank r owns envs [r*N_local, (r+1)*N_local) of the global N = world * N_local and
steps them (rollout, GAE, normalisation are per env: no communication).  Exchange: ONE all-reduce
(SUM) of the flat actor+critic gradient per optimizer step; every rank then runs the identical
fused Adam, so replicas stay bit-identical.

Two minibatch modes:
  "local" (weak scaling, the bench): each rank shuffles its own N_local*T rows and takes B rows
          per minibatch; the loss is scaled by 1/(B*world) so the summed gradient is the mean over
          the global B*world rows.
  "exact": every rank draws the SAME global permutation of N*T rows (reference order,
          ppo.py:103-106), keeps the rows that fall in its shard (compacted on device) and scales
          by 1/B: after the all-reduce the gradient equals the single-process reference gradient
          up to summation order.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def shard_range(n_global: int, world: int, rank: int) -> Tuple[int, int]:
    """Env range of ``rank`` (equal shards; N must divide evenly)."""
    if n_global % world:
        raise ValueError(f"num_envs={n_global} is not divisible by world size {world}")
    n = n_global // world
    return rank * n, (rank + 1) * n


class DataParallel:
    """Rank/world bookkeeping + the one gradient exchange."""

    def __init__(self, process_group=None, mode: str = "local"):
        if mode not in ("local", "exact"):
            raise ValueError(f"unknown data-parallel mode {mode!r}")
        self.pg = process_group
        self.mode = mode
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            self.world = torch.distributed.get_world_size(process_group)
            self.rank = torch.distributed.get_rank(process_group)
        else:
            self.world, self.rank = 1, 0
        # PPO_DP_REHEARSE=1: one rank runs the data-parallel step sequence (eager launches, the
        # gradient folded to HBM, the separate Adam / gather tail) with a no-op exchange -- the
        # DP kernel cost measured without a second process contending for the GPU
        import os
        # Only the kernel sequence follows it (``active``); the RNG streams and the loss scale
        # follow ``world`` alone, so the rehearsal computes what the single-rank run computes.
        self.rehearse = self.world == 1 and os.environ.get("PPO_DP_REHEARSE") == "1"
        if self.rehearse:
            import warnings
            warnings.warn("PPO_DP_REHEARSE=1: running the data-parallel kernel sequence (eager, "
                          "no hipGraphs) with a no-op exchange on one rank", stacklevel=2)

    @property
    def active(self) -> bool:
        """The data-parallel kernel sequence (fold to HBM, exchange, separate Adam tail) runs."""
        return self.world > 1 or self.rehearse

    def allreduce_grad(self, flat_grad: torch.Tensor) -> None:
        """SUM of the flat gradient over ranks, in place, ordered on the current stream (RCCL
        runs it on its own stream; the compute stream waits on it, the host does not).  There is
        no asynchronous form: nothing independent sits between the gradient and its use -- Adam
        consumes the sum and the next minibatch's forward consumes Adam's weights."""
        if self.world > 1:
            torch.distributed.all_reduce(flat_grad, op=torch.distributed.ReduceOp.SUM,
                                         group=self.pg)

    def broadcast_params(self, flat: torch.Tensor, src: int = 0) -> None:
        """Start every replica from rank ``src``'s parameters."""
        if self.world > 1:
            torch.distributed.broadcast(flat, src=src, group=self.pg)

    def loss_scale(self, b_local: int) -> int:
        """Global minibatch size the per-row loss terms are divided by."""
        return b_local if self.mode == "exact" else b_local * self.world

    def global_envs(self, n_local: int) -> int:
        return n_local * self.world

    def my_shard(self, n_local: int) -> Tuple[int, int]:
        return shard_range(n_local * self.world, self.world, self.rank)


def maybe_init_from_env(backend: Optional[str] = None) -> None:
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*), if present."""
    import os
    if torch.distributed.is_initialized() or int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    torch.distributed.init_process_group(backend)
