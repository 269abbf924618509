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

The exchange (RCCL process groups, i.e. the ``nccl`` backend on ROCm): a native communicator owned
by the engine library (csrc/comm.hip, ``ppo_comm_*`` / ``ppo_allreduce_grads``), created once from
a unique id that rank 0 broadcasts over the process group.  Its all-reduce is issued on the compute
stream, so the whole optimizer loop -- fused gradient, all-reduce, Adam tail -- is captured in ONE
hipGraph and replayed ("a persistent RCCL comm and a HIP-graph-captured
all-reduce").  gloo process groups (CPU tests) keep torch.distributed.all_reduce, eagerly.
"""
from __future__ import annotations

import os
import warnings
from typing import Optional, Tuple

import torch


def shard_range(n_global: int, world: int, rank: int) -> Tuple[int, int]:
    """Env range of ``rank`` (equal shards; N must divide evenly)."""
    if n_global % world:
        raise ValueError(f"num_envs={n_global} is not divisible by world size {world}")
    n = n_global // world
    return rank * n, (rank + 1) * n


class NativeComm:
    """One ``ppo_comm`` (csrc/comm.hip): an RCCL communicator over the ranks of ``process_group``
    on ``device``.  ``allreduce`` sums an f32 tensor in place on the current stream (capturable)."""

    def __init__(self, process_group, device: torch.device, world: int, rank: int):
        import ctypes
        from . import _lib
        self.lib = _lib.load()
        self.device = torch.device(device)
        self.world, self.rank = world, rank
        uid = torch.zeros(_lib.COMM_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
            _lib.check(self.lib.ppo_comm_unique_id(buf))
            uid.copy_(torch.frombuffer(bytearray(bytes(buf)), dtype=torch.uint8))
        if world > 1:  # the one use of the process group: the id from rank 0
            on_dev = torch.distributed.get_backend(process_group) == "nccl"
            t = uid.to(self.device) if on_dev else uid
            torch.distributed.broadcast(t, src=0, group=process_group)
            uid = t.cpu()
        arr = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)(*uid.tolist())
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.ppo_comm_create(arr, world, rank, self.device.index or 0,
                                                ctypes.byref(handle)))
        self._comm = handle

    @property
    def handle(self):
        return self._comm

    def allreduce(self, t: torch.Tensor) -> None:
        from . import _lib
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
            raise ValueError("NativeComm.allreduce: contiguous f32 tensor on the comm's device")
        _lib.check(self.lib.ppo_comm_allreduce(self._comm, t.data_ptr(), t.numel(),
                                               torch.cuda.current_stream(self.device).cuda_stream))

    def check(self) -> None:
        from . import _lib
        _lib.check(self.lib.ppo_comm_check(self._comm))

    def close(self) -> None:
        if getattr(self, "_comm", None) is not None and self._comm.value:
            self.lib.ppo_comm_destroy(self._comm)
        self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


class DataParallel:
    """Rank/world bookkeeping + the one gradient exchange."""

    def __init__(self, process_group=None, mode: str = "local"):
        if mode not in ("local", "exact"):
            raise ValueError(f"unknown data-parallel mode {mode!r}")
        self.pg = process_group
        self.mode = mode
        self.comm: Optional[NativeComm] = None
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            self.world = torch.distributed.get_world_size(process_group)
            self.rank = torch.distributed.get_rank(process_group)
            self.backend = torch.distributed.get_backend(process_group)
        else:
            self.world, self.rank, self.backend = 1, 0, None
        # PPO_DP_REHEARSE: one rank runs the data-parallel step sequence (the gradient folded to
        # HBM, the exchange, the separate Adam / gather tail) -- the DP kernel cost measured
        # without a second process contending for the GPU.  "1": a no-op exchange, eager launches;
        # "rccl" (needs a world-1 nccl process group): the real native RCCL all-reduce, the loop
        # captured in a hipGraph exactly as at world > 1.
        # Only the kernel sequence follows it (``active``); the RNG streams and the loss scale
        # follow ``world`` alone, so the rehearsal computes what the single-rank run computes.
        rehearse = os.environ.get("PPO_DP_REHEARSE", "")
        self.rehearse = self.world == 1 and rehearse in ("1", "rccl")
        self.rehearse_rccl = self.rehearse and rehearse == "rccl"
        if self.rehearse_rccl and self.backend != "nccl":
            raise RuntimeError("PPO_DP_REHEARSE=rccl needs an initialised nccl process group")
        if self.rehearse:
            how = ("native RCCL exchange, graph-captured" if self.rehearse_rccl
                   else "no-op exchange, eager")
            warnings.warn(f"PPO_DP_REHEARSE={rehearse}: running the data-parallel kernel sequence "
                          f"on one rank ({how})", stacklevel=2)

    @property
    def active(self) -> bool:
        """The data-parallel kernel sequence (fold to HBM, exchange, separate Adam tail) runs."""
        return self.world > 1 or self.rehearse

    @property
    def graph_safe(self) -> bool:
        """The exchange can sit inside a hipGraph capture: the native RCCL communicator, or no
        exchange at all (one rank)."""
        return self.comm is not None or self.world == 1

    def attach(self, engine, device: torch.device) -> None:
        """Create the native communicator for an RCCL process group (or the rccl rehearsal) and
        hand it to the engine's ctx (``ppo_ctx_set_comm``).  The logged actor
        loss carries the entropy bonus on rank 0 only, so the per-rank losses sum to the
        reference's (ppo.py:128-132)."""
        if self.world > 1 and hasattr(engine, "loss_entropy_share"):
            engine.loss_entropy_share(1.0 if self.rank == 0 else 0.0)
        if self.comm is None and (self.backend == "nccl" and (self.world > 1 or self.rehearse_rccl)):
            if os.environ.get("PPO_DP_NATIVE", "1") == "1":
                try:
                    self.comm = NativeComm(self.pg, device, self.world, self.rank)
                except RuntimeError as err:  # _lib.EngineError: no usable RCCL in this process
                    warnings.warn(f"native RCCL communicator unavailable ({err}); the gradient "
                                  f"all-reduce goes through torch.distributed, eagerly")
                    self.comm = None
        if self.comm is not None and hasattr(engine, "set_comm"):
            engine.set_comm(self.comm)

    def allreduce_grad(self, flat_grad: torch.Tensor) -> None:
        """SUM of the flat gradient over ranks, in place, ordered on the current stream (the native
        RCCL all-reduce runs on it; torch.distributed's runs on its own stream that the compute
        stream waits on).  The host does not block.  There is no asynchronous form: nothing
        independent sits between the gradient and its use -- Adam consumes the sum and the next
        minibatch's forward consumes Adam's weights."""
        if self.comm is not None:
            self.comm.allreduce(flat_grad)
        elif self.world > 1:
            torch.distributed.all_reduce(flat_grad, op=torch.distributed.ReduceOp.SUM,
                                         group=self.pg)

    def allreduce_log(self, t: torch.Tensor) -> None:
        """SUM for logging (once per iteration): the process group's own collective."""
        if self.world > 1:
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM, group=self.pg)

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
