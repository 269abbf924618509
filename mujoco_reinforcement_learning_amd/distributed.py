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


class NativeCommUnavailable(RuntimeError):
    """Raised on EVERY rank when any rank cannot take part in the native communicator (the ranks
    agree on it before and after ncclCommInitRank, so no rank is left inside a collective the
    others skipped)."""


def _resolve_device(device) -> torch.device:
    """An indexed CUDA device: ``cuda`` without an index means the current device (an
    unindexed device used to put every rank's communicator on GPU 0)."""
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


class NativeComm:
    """One ``ppo_comm`` (csrc/comm.hip): an RCCL communicator over ``world`` ranks on ``device``,
    built from a unique id every rank already holds.  ``allreduce`` sums an f32 tensor in place on
    the current stream (capturable).  Use ``DataParallel.attach`` to build one: it agrees on the id
    and on the outcome across ranks."""

    def __init__(self, uid: bytes, device: torch.device, world: int, rank: int):
        import ctypes
        from . import _lib
        self.lib = _lib.load()
        self.device = _resolve_device(device)
        self.world, self.rank = world, rank
        self._retired = False
        arr = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)(*uid)
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.ppo_comm_create(arr, world, rank, self.device.index,
                                                ctypes.byref(handle)))
        self._comm = handle

    @property
    def handle(self):
        return self._comm

    def info(self) -> dict:
        """What the communicator itself reports (ppo_comm_query: ncclCommCount / ncclCommUserRank /
        its device), for the bench line -- not what the caller asked for."""
        import ctypes
        from . import _lib
        nranks, rank, device = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.ppo_comm_query(self._comm, ctypes.byref(nranks), ctypes.byref(rank),
                                           ctypes.byref(device)))
        return {"nranks": nranks.value, "rank": rank.value, "device": device.value,
                "rccl_version": int(self.lib.ppo_comm_version())}

    def allreduce(self, t: torch.Tensor) -> None:
        from . import _lib
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
            raise ValueError("NativeComm.allreduce: contiguous f32 tensor on the comm's device")
        _lib.check(self.lib.ppo_comm_allreduce(self._comm, t.data_ptr(), t.numel(),
                                               torch.cuda.current_stream(self.device).cuda_stream))

    def check(self) -> None:
        from . import _lib
        _lib.check(self.lib.ppo_comm_check(self._comm))

    def retire(self) -> None:
        """Stop using this communicator WITHOUT ncclCommDestroy: after a failed graph capture its
        state on some rank may hold a half-recorded collective, and a destroy that waits on it
        would block; the handle is left to the process's exit."""
        self._retired = True

    def close(self) -> None:
        if getattr(self, "_comm", None) is not None and self._comm.value and not self._retired:
            self.lib.ppo_comm_destroy(self._comm)
        self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


def _native_unique_id() -> bytes:
    """rank 0's RCCL unique id (ppo_comm_unique_id); raises the engine's error when RCCL is absent."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    _lib.check(lib.ppo_comm_unique_id(buf))
    return bytes(buf)


def _native_loadable() -> bool:
    """RCCL resolvable in this process (ppo_comm_version > 0), checked before any rank commits to
    the collective ncclCommInitRank."""
    from . import _lib
    try:
        return int(_lib.load().ppo_comm_version()) > 0
    except Exception:  # noqa: BLE001 -- any failure to load means "not available here"
        return False


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

    def agree(self, ok: bool) -> bool:
        """True only if ``ok`` holds on every rank: a MIN all-reduce of one flag over the process
        group (its own collective, not the native communicator).  Every decision that changes
        which collectives a rank issues goes through this, so all ranks take the same branch."""
        if self.world <= 1 or not torch.distributed.is_initialized():
            return bool(ok)
        dev = (torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl"
               else torch.device("cpu"))
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN, group=self.pg)
        return bool(int(t.item()))

    def _broadcast_id(self, ok: bool, uid: bytes) -> Tuple[bool, bytes]:
        """rank 0's (ok, unique id) to every rank: one flag byte + the id, so a rank 0 that could
        not draw an id sends a sentinel instead of leaving the others blocked in the broadcast."""
        from . import _lib
        n = _lib.COMM_ID_BYTES
        t = torch.zeros(n + 1, dtype=torch.uint8)
        if self.rank == 0:
            t[0] = 1 if ok else 0
            if ok:
                t[1:] = torch.frombuffer(bytearray(uid), dtype=torch.uint8)
        if self.world > 1:
            on_dev = self.backend == "nccl"
            w = t.to(torch.device("cuda", torch.cuda.current_device())) if on_dev else t
            torch.distributed.broadcast(w, src=0, group=self.pg)
            t = w.cpu()
        return bool(t[0]), bytes(t[1:].tolist())

    def build_comm(self, device, make_id=None, make_comm=None, loadable=None):
        """The native communicator, built only if every rank can build it (NativeCommUnavailable on
        every rank otherwise -- the same outcome everywhere):
          1. every rank checks that RCCL resolves here; rank 0 draws the unique id;
          2. rank 0 broadcasts (ok, id) -- a sentinel when it failed;
          3. agree(all loadable and rank 0 ok), else every rank gives up before the collective init;
          4. ncclCommInitRank on every rank; agree(all succeeded), else the ranks that did build one
             retire it and every rank gives up.
        ``make_id`` / ``make_comm`` / ``loadable`` are injectable for the CPU tests."""
        make_id = make_id or _native_unique_id
        make_comm = make_comm or (lambda uid, dev, w, r: NativeComm(uid, dev, w, r))
        loadable = loadable or _native_loadable
        local_ok = bool(loadable())
        uid, id_ok, why = b"", True, ""
        if self.rank == 0:
            try:
                uid = make_id()
            except RuntimeError as err:
                id_ok, why = False, f"rank 0 could not draw the RCCL unique id: {err}"
        id_ok, uid = self._broadcast_id(id_ok, uid)
        if not self.agree(local_ok and id_ok):
            raise NativeCommUnavailable(why or ("RCCL is not resolvable on some rank" if id_ok else
                                                "rank 0 could not draw the RCCL unique id"))
        comm, err_msg = None, ""
        try:
            comm = make_comm(uid, device, self.world, self.rank)
        except RuntimeError as err:
            err_msg = str(err)
        if not self.agree(comm is not None):
            if comm is not None:
                comm.retire()
            raise NativeCommUnavailable(err_msg or "ncclCommInitRank failed on another rank")
        return comm

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
                    self.comm = self.build_comm(_resolve_device(device))
                except NativeCommUnavailable as err:  # the same on every rank (build_comm)
                    warnings.warn(f"native RCCL communicator unavailable ({err}); the gradient "
                                  f"all-reduce goes through torch.distributed, eagerly")
                    self.comm = None
        if self.comm is not None and hasattr(engine, "set_comm"):
            engine.set_comm(self.comm)

    def drop_native(self, engine=None) -> None:
        """Every rank leaves the native communicator together (after agree() said some rank
        could not use it): the engine's ctx is detached, the communicator retired, and the
        exchange falls back to torch.distributed."""
        if engine is not None and hasattr(engine, "set_comm"):
            engine.set_comm(None)
        if self.comm is not None:
            self.comm.retire()
        self.comm = None

    def capture_agreed(self, capture, engine=None) -> Optional[str]:
        """Run ``capture()`` (recording an update loop that contains the native all-reduce into a
        hipGraph).  None when it succeeded on EVERY rank.  When it failed on any rank, every rank
        leaves the native communicator (drop_native) and the reason is returned, so all ranks
        continue on the same eager torch.distributed path (the fallback used to be
        decided per rank).  Without a native communicator a capture failure is a plain error."""
        err = None
        try:
            capture()
        except RuntimeError as e:
            if self.comm is None:
                raise
            err = str(e) or type(e).__name__
        if self.agree(err is None):
            return None
        self.drop_native(engine)
        return err or "the capture failed on another rank"

    def comm_info(self) -> dict:
        """{backend, native, nranks, ...} of the exchange as it will run: read back from the native
        communicator when there is one, else the process group's own size."""
        out = {"backend": self.backend or "none", "native": self.comm is not None,
               "nranks": self.world, "rank": self.rank}
        if self.comm is not None and hasattr(self.comm, "info"):
            out.update(self.comm.info())
        return out

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
