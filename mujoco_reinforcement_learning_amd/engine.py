"""Torch-tensor front end of the C-ABI: ``Engine`` owns one ``ppo_ctx`` per (process, GPU).

Every call launches on ``torch.cuda.current_stream()`` and validates shapes/dtypes on the host
before handing raw pointers to the library (include/ppo_engine.h); errors surface as
``EngineError`` (a RuntimeError) carrying ``ppo_last_error()``.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from . import _lib
from ._lib import check, ptr

HUMANOID_SLICE_EDGES = (0, 22, 45, 175, 253, 270)  # running_gym_sequential_vectorized.py:70-80


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _need(t: torch.Tensor, name: str, dtype=None, shape=None, device=None):
    if t is None:
        raise ValueError(f"{name} is required")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (got {t.device})")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise RuntimeError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
    return t


def slice_edges(obs_dim: int) -> list:
    """The reference's Humanoid slices clipped to O, as ascending edges (python slice semantics)."""
    edges = [min(e, obs_dim) for e in HUMANOID_SLICE_EDGES] + [obs_dim]
    return edges


class Engine:
    """One ``ppo_ctx``: network shapes + activation workspace + split-K slabs on one GPU."""

    def __init__(self, obs_dim: int, window: int, act_dim: int, actor_hidden: Sequence[int],
                 critic_hidden: Sequence[int], activation: str = "relu",
                 actor_use_bias: bool = True, output_max_value: float = 1.0,
                 max_rows: int = 65536, device: Optional[torch.device] = None):
        self.lib = _lib.load()
        if activation not in _lib.ACT_CODES:
            raise ValueError(f"unsupported activation {activation!r}; use one of "
                             f"{sorted(_lib.ACT_CODES)}")
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        cfg = _lib.NetCfg()
        cfg.obs_dim, cfg.window, cfg.act_dim = obs_dim, window, act_dim
        cfg.activation = _lib.ACT_CODES[activation]
        cfg.actor_use_bias = int(bool(actor_use_bias))
        cfg.n_actor_hidden = len(actor_hidden)
        cfg.n_critic_hidden = len(critic_hidden)
        for i, h in enumerate(actor_hidden):
            cfg.actor_hidden[i] = int(h)
        for i, h in enumerate(critic_hidden):
            cfg.critic_hidden[i] = int(h)
        cfg.output_max_value = float(output_max_value)
        cfg.max_rows = int(max_rows)
        self.cfg = cfg
        self.obs_dim, self.window, self.act_dim = obs_dim, window, act_dim
        self.in_dim = obs_dim * window
        self.max_rows = int(max_rows)
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self.lib.ppo_ctx_create(ctypes.byref(cfg), self.device.index or 0,
                                          ctypes.byref(handle)))
        self._ctx = handle
        self.n_actor = int(self.lib.ppo_param_count(self._ctx, 0))
        self.n_critic = int(self.lib.ppo_param_count(self._ctx, 1))
        self.n_params = int(self.lib.ppo_param_count(self._ctx, -1))
        self._params = None
        self.precision = "f32"

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            try:
                self.lib.ppo_ctx_destroy(ctx)
            except Exception:  # interpreter shutdown
                pass
            self._ctx = None

    # ---- parameters ----------------------------------------------------------------------
    def param_offsets(self) -> list:
        """Flat offset of every parameter tensor (torch parameters() order, actor then critic)."""
        n = self.lib.ppo_param_offsets(self._ctx, None, 0)
        arr = (ctypes.c_int64 * n)()
        self.lib.ppo_param_offsets(self._ctx, arr, n)
        return list(arr)

    def bind(self, flat_params: torch.Tensor) -> None:
        _need(flat_params, "flat_params", torch.float32, (self.n_params,), self.device)
        check(self.lib.ppo_bind_params(self._ctx, ptr(flat_params)))
        self._params = flat_params

    # ---- A2-A4 ---------------------------------------------------------------------------
    def policy_step(self, state: torch.Tensor, eps: Optional[torch.Tensor] = None, seed: int = 0,
                    offset: int = 0, action=None, logp=None, value=None, mean=None) -> None:
        n = state.shape[0]
        _need(state, "state", torch.float32, device=self.device)
        if state.numel() != n * self.in_dim:
            raise RuntimeError(f"state has {state.numel() // max(n, 1)} features per row, "
                               f"expected W*O={self.in_dim}")
        if eps is not None:
            _need(eps, "eps", torch.float32, (n, self.act_dim), self.device)
        for name, t, shp in (("action", action, (n, self.act_dim)), ("logp", logp, (n,)),
                             ("value", value, (n,)), ("mean", mean, (n, self.act_dim))):
            if t is not None:
                _need(t, name, torch.float32, device=self.device)
                if t.numel() != n * (shp[1] if len(shp) == 2 else 1):
                    raise RuntimeError(f"{name} has {t.numel()} elements, expected shape {shp}")
        check(self.lib.ppo_policy_step(self._ctx, ptr(state), n, ptr(eps), seed, offset,
                                       ptr(action), ptr(logp), ptr(value), ptr(mean),
                                       _stream(self.device)))

    def set_comm(self, comm) -> None:
        """Attach a ``distributed.NativeComm`` to the ctx (``ppo_ctx_set_comm``); None detaches."""
        check(self.lib.ppo_ctx_set_comm(self._ctx, None if comm is None else comm.handle))
        self._comm = comm  # the ctx does not own it: keep it alive as long as the ctx uses it

    def allreduce_grads(self, flat_grad: torch.Tensor) -> None:
        """``ppo_allreduce_grads``: SUM of the flat gradient over the attached
        communicator's ranks, in place, on the current stream."""
        _need(flat_grad, "flat_grad", torch.float32, (self.n_params,), self.device)
        check(self.lib.ppo_allreduce_grads(self._ctx, ptr(flat_grad), flat_grad.numel(),
                                           _stream(self.device)))

    def loss_entropy_share(self, share: float) -> None:
        """Share of the entropy bonus in the LOGGED actor loss (ppo_ctx_loss_entropy_share)."""
        check(self.lib.ppo_ctx_loss_entropy_share(self._ctx, float(share)))

    def pack_weights(self) -> None:
        """Refresh the bf16 weight images of the fused kernels from the bound parameters (after
        an optimizer step, before a rollout).  No-op outside the fused bf16 path."""
        check(self.lib.ppo_pack_weights(self._ctx, _stream(self.device)))

    def observe_act(self, window: torch.Tensor, state: torch.Tensor, obs: Optional[torch.Tensor] = None,
                    reset: Optional[torch.Tensor] = None, all_reset: bool = False,
                    normalize: bool = True, eps: Optional[torch.Tensor] = None, seed: int = 0,
                    offset: int = 0, action=None, logp=None, value=None, mean=None) -> None:
        """A1-A4 for one rollout step (ppo_observe_act): push ``obs`` (N, O) f64 into ``window``
        (N, O, W) f64 (in place; skipped when obs is None), standardise into ``state`` (N, W*O)
        f32, then sample / evaluate like :meth:`policy_step`."""
        n, o, w = window.shape
        _need(window, "window", torch.float64, device=self.device)
        if (o, w) != (self.obs_dim, self.window):
            raise RuntimeError(f"window is {(o, w)}, expected (O, W) = {(self.obs_dim, self.window)}")
        _need(state, "state", torch.float32, device=self.device)
        if state.numel() != n * o * w:
            raise RuntimeError(f"state must hold (N, W*O) = {(n, o * w)} floats")
        if obs is not None:
            _need(obs, "obs", torch.float64, (n, o), self.device)
        if reset is not None:
            _need(reset, "reset", None, (n,), self.device)
        if eps is not None:
            _need(eps, "eps", torch.float32, (n, self.act_dim), self.device)
        for name, t, k in (("action", action, self.act_dim), ("logp", logp, 1), ("value", value, 1),
                           ("mean", mean, self.act_dim)):
            if t is not None:
                _need(t, name, torch.float32, device=self.device)
                if t.numel() != n * k:
                    raise RuntimeError(f"{name} has {t.numel()} elements, expected {n * k}")
        edges = slice_edges(o)
        arr = (ctypes.c_int32 * len(edges))(*edges)
        check(self.lib.ppo_observe_act(self._ctx, ptr(window), ptr(obs), ptr(reset),
                                       int(all_reset), arr, len(edges) - 1, int(normalize),
                                       ptr(state), n, ptr(eps), seed, offset, ptr(action),
                                       ptr(logp), ptr(value), ptr(mean), _stream(self.device)))

    def host_rollout(self, desc, window: torch.Tensor, normalize: bool, states, actions, logp,
                     values, reward, terminated, obs_next, eps: Optional[torch.Tensor], seed: int,
                     base_offset: int) -> None:
        """The whole pipelined host-physics rollout in one native call (ppo_host_rollout): per
        step and worker group, observe + act, action D2H, worker release / wait and result H2D
        from one host thread.  ``desc`` is the pool's ``_lib.HostPoolDesc`` (gen updated in
        place); the buffers are the rollout buffer's time-major arrays."""
        n, o, w = window.shape
        t = actions.shape[0]
        _need(window, "window", torch.float64, device=self.device)
        _need(states, "states", torch.float32, device=self.device)
        _need(actions, "actions", torch.float32, (t, n, self.act_dim), self.device)
        _need(logp, "logp", torch.float32, (t, n), self.device)
        _need(values, "values", torch.float32, (t + 1, n), self.device)
        _need(reward, "reward", torch.float64, (t, n), self.device)
        _need(terminated, "terminated", None, (t, n), self.device)
        _need(obs_next, "obs_next", torch.float64, (n, o), self.device)
        if states.numel() != (t + 1) * n * o * w:
            raise RuntimeError("states must hold (T+1, N, W*O) floats")
        if eps is not None:
            _need(eps, "eps", torch.float32, (t, n, self.act_dim), self.device)
        edges = slice_edges(o)
        arr = (ctypes.c_int32 * len(edges))(*edges)
        check(self.lib.ppo_host_rollout(
            self._ctx, ctypes.byref(desc), ptr(window), arr, len(edges) - 1, int(normalize),
            ptr(states), ptr(actions), ptr(logp), ptr(values), ptr(reward), ptr(terminated),
            ptr(obs_next), n, o, w, self.act_dim, t, ptr(eps), seed, base_offset,
            _stream(self.device)))

    def set_precision(self, precision: str) -> None:
        """GEMM precision: "f32" (parity with the reference, default) or "bf16" (bf16 operands,
        f32 accumulation; activations, params and optimizer state stay f32)."""
        if precision not in _lib.PREC_CODES:
            raise ValueError(f"unknown precision {precision!r}; use one of {sorted(_lib.PREC_CODES)}")
        check(self.lib.ppo_ctx_set_precision(self._ctx, _lib.PREC_CODES[precision]))
        self.precision = precision

    def set_rng_counter(self, counter: Optional[torch.Tensor]) -> None:
        """Philox offset base read on the device at kernel run time (int64 scalar tensor on this
        device, or None): lets a graph-captured rollout replay with fresh noise."""
        if counter is not None:
            _need(counter, "counter", torch.int64, (1,), self.device)
        check(self.lib.ppo_ctx_set_rng_counter(self._ctx, ptr(counter)))
        self._rng_counter = counter  # keep the buffer alive while the ctx may read it

    def fused_direct(self, enable: Optional[bool] = None) -> bool:
        """ppo_ctx_fused_direct: the 8-wave fused kernel reads the staged records through the row
        indices itself (True, default) or the gathered copy (False); returns the current mode."""
        if enable is not None:
            check(self.lib.ppo_ctx_fused_direct(self._ctx, int(bool(enable))))
        return bool(self.lib.ppo_ctx_fused_direct(self._ctx, -1))

    # ---- measurement ---------------------------------------------------------------------
    def timing(self, enable: bool, capacity: int = 65536) -> None:
        """Record a HIP event pair around every kernel this context launches (live roofline)."""
        check(self.lib.ppo_ctx_timing(self._ctx, int(enable), int(capacity)))

    def timing_read(self) -> dict:
        """{class: {"ms": total kernel ms, "launches": n, "flops": algorithmic, "bytes": ...}}"""
        out = {}
        n_cls = self.lib.ppo_ctx_timing_read(self._ctx, -1, None, None, None, None)
        for c in range(n_cls):
            ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            cnt = ctypes.c_int64()
            check(self.lib.ppo_ctx_timing_read(self._ctx, c, ctypes.byref(ms), ctypes.byref(cnt),
                                               ctypes.byref(fl), ctypes.byref(by)))
            name = self.lib.ppo_kernel_class_name(c).decode()
            out[name] = {"ms": ms.value, "launches": cnt.value, "flops": fl.value,
                         "bytes": by.value}
        return out

    def phase_stamps(self, enable: bool):
        """Diagnostics: enable=True stamps the fused kernel's phases; enable=False returns the
        last launch's per-phase cycle sums as a (2, G, 13) uint64 tensor (ppo_ctx_phase_stamps;
        slots 10/11 prologue/epilogue cycles, 12 the body's 100 MHz realtime ticks)."""
        if enable:
            check(self.lib.ppo_ctx_phase_stamps(self._ctx, 1, None, 0))
            return None
        out = torch.zeros(2 * 128 * 13, dtype=torch.int64)
        n = self.lib.ppo_ctx_phase_stamps(self._ctx, 0, ctypes.c_void_p(out.data_ptr()), out.numel())
        check(min(n, 0))
        return out[:n].view(2, -1, 13)

    def timing_kernels(self) -> dict:
        """Same records per kernel instantiation, keyed by the rocprofv3 kernel name:
        {name: {"class": ..., "ms", "launches", "flops", "bytes"}}."""
        out = {}
        n_k = self.lib.ppo_ctx_timing_kernel(self._ctx, -1, None, None, None, None, None, None)
        check(min(n_k, 0))
        for i in range(n_k):
            name, cls = ctypes.c_char_p(), ctypes.c_int()
            ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            cnt = ctypes.c_int64()
            check(self.lib.ppo_ctx_timing_kernel(self._ctx, i, ctypes.byref(name),
                                                 ctypes.byref(cls), ctypes.byref(ms),
                                                 ctypes.byref(cnt), ctypes.byref(fl),
                                                 ctypes.byref(by)))
            out[name.value.decode()] = {
                "class": self.lib.ppo_kernel_class_name(cls.value).decode(), "ms": ms.value,
                "launches": cnt.value, "flops": fl.value, "bytes": by.value}
        return out

    # ---- A11-A13 -------------------------------------------------------------------------
    def minibatch_grad(self, states, actions, old_logp, adv, vtarget, rows, b: int, grad, loss,
                       clip_lo: float, clip_hi: float, entropy_coef: float, inv_b: float,
                       inv_ba: float, count: Optional[torch.Tensor] = None) -> None:
        _need(rows, "rows", torch.int32, device=self.device)
        _need(grad, "grad", torch.float32, (self.n_params,), self.device)
        _need(loss, "loss", torch.float32, device=self.device)
        if loss.numel() != 2:
            raise RuntimeError("loss must hold 2 floats")
        check(self.lib.ppo_minibatch_grad(
            self._ctx, ptr(states), ptr(actions), ptr(old_logp), ptr(adv), ptr(vtarget),
            ptr(rows), int(b), ptr(count), clip_lo, clip_hi, entropy_coef, inv_b, inv_ba,
            ptr(grad), ptr(loss), _stream(self.device)))

    # ---- staged minibatch path (fused bf16 engine) ---------------------------------------
    @property
    def fused(self) -> bool:
        """True when the fused bf16 kernels run (precision bf16, two equal hidden layers of a
        compiled width, W*O <= 32, A <= 8): the staged path below is available."""
        return bool(self.lib.ppo_ctx_fused_active(self._ctx))

    def stage_records(self, states, actions, old_logp, adv, vtarget) -> None:
        """Pack the time-major storage arrays (rows = T*N) into the ctx's 128 B per-row records
        that minibatch_grad_staged gathers (once per iteration, after GAE)."""
        n_rows = old_logp.numel()
        for name, t in (("states", states), ("actions", actions), ("old_logp", old_logp),
                        ("adv", adv), ("vtarget", vtarget)):
            _need(t, name, torch.float32, None, self.device)
            width = t.shape[-1] if name in ("states", "actions") else 1
            if t.numel() < n_rows * width:  # states may carry the extra slot T
                raise RuntimeError(f"{name}: {t.numel()} elements for {n_rows} rows x {width}")
        check(self.lib.ppo_stage_records(self._ctx, ptr(states), ptr(actions), ptr(old_logp),
                                         ptr(adv), ptr(vtarget), int(n_rows),
                                         _stream(self.device)))

    def gae_stage_records(self, value, next_value, reward, terminated, gamma: float, lmbda: float,
                          adv, vtarget, states, actions, old_logp, done=None,
                          force_last_done: bool = True) -> None:
        """gae(...) and stage_records(states, actions, old_logp, adv, vtarget) in one pass
        (ppo_gae_stage_records); only valid when adv / vtarget are not normalised in between."""
        t, n = value.shape[0], value.shape[1]
        _gae_check(value, next_value, reward, terminated, adv, vtarget, done)
        for name, x, width in (("states", states, self.obs_dim * self.window),
                               ("actions", actions, self.act_dim), ("old_logp", old_logp, 1)):
            _need(x, name, torch.float32, None, self.device)
            if x.numel() < t * n * width:  # states may carry the extra slot T
                raise RuntimeError(f"{name}: {x.numel()} elements for {t * n} rows x {width}")
        check(self.lib.ppo_gae_stage_records(
            self._ctx, ptr(value), ptr(next_value), ptr(reward), int(reward.dtype == torch.float64),
            ptr(done), ptr(terminated), int(force_last_done), n, t, float(gamma), float(lmbda),
            ptr(adv), ptr(vtarget), ptr(states), ptr(actions), ptr(old_logp),
            _stream(self.device)))

    def minibatch_grad_staged(self, rows, b: int, grad, loss, clip_lo: float, clip_hi: float,
                              entropy_coef: float, inv_b: float, inv_ba: float,
                              count: Optional[torch.Tensor] = None,
                              weights_current: bool = False, rows_gathered: bool = False) -> None:
        """minibatch_grad on the staged records; weights_current=True skips the bf16 weight
        refresh (valid right after adam_pack), rows_gathered=True the row gather (the previous
        adam_pack(next_rows=rows) did it)."""
        _need(rows, "rows", torch.int32, device=self.device)
        _need(grad, "grad", torch.float32, (self.n_params,), self.device)
        _need(loss, "loss", torch.float32, device=self.device)
        if loss.numel() != 2:
            raise RuntimeError("loss must hold 2 floats")
        check(self.lib.ppo_minibatch_grad_staged(
            self._ctx, ptr(rows), int(b), ptr(count), clip_lo, clip_hi, entropy_coef, inv_b,
            inv_ba, ptr(grad), ptr(loss), (1 if weights_current else 0) | (2 if rows_gathered else 0),
            _stream(self.device)))

    def update_step_staged(self, rows, b: int, grad, loss, m, v, clip_lo: float, clip_hi: float,
                           entropy_coef: float, inv_b: float, inv_ba: float,
                           sched: Optional[torch.Tensor] = None, neg_step_actor: float = 0.0,
                           neg_step_critic: float = 0.0, bc2_sqrt: float = 1.0,
                           one_minus_beta1: float = 0.1, beta2: float = 0.999,
                           one_minus_beta2: float = 0.001, eps: float = 1e-8,
                           next_rows: Optional[torch.Tensor] = None, weights_current: bool = False,
                           rows_gathered: bool = False) -> None:
        """One optimizer step on the staged records (single rank): minibatch_grad_staged, then
        adam_pack, with the next minibatch's row gather (next_rows) folded into the last launch.
        rows_gathered=True: the previous step's next_rows were these rows."""
        _need(rows, "rows", torch.int32, device=self.device)
        for name, t in (("grad", grad), ("m", m), ("v", v)):
            _need(t, name, torch.float32, (self.n_params,), self.device)
        _need(loss, "loss", torch.float32, device=self.device)
        if loss.numel() != 2:
            raise RuntimeError("loss must hold 2 floats")
        if sched is not None:
            _need(sched, "sched", torch.float32, None, self.device)
        nb = 0
        if next_rows is not None:
            _need(next_rows, "next_rows", torch.int32, device=self.device)
            nb = next_rows.numel()
        flags = (1 if weights_current else 0) | (2 if rows_gathered else 0)
        check(self.lib.ppo_update_step_staged(
            self._ctx, ptr(rows), int(b), ptr(next_rows), nb, clip_lo, clip_hi, entropy_coef,
            inv_b, inv_ba, ptr(grad), ptr(loss), ptr(m), ptr(v), ptr(sched), neg_step_actor,
            neg_step_critic, bc2_sqrt, one_minus_beta1, beta2, one_minus_beta2, eps, flags,
            _stream(self.device)))

    def gather_staged_rows(self, rows) -> None:
        """ppo_gather_staged_rows: the minibatch's rows from the staged records into the gathered
        workspace (read by minibatch_grad_staged(rows_gathered=True))."""
        _need(rows, "rows", torch.int32, device=self.device)
        check(self.lib.ppo_gather_staged_rows(self._ctx, ptr(rows), rows.numel(),
                                              _stream(self.device)))

    def adam_pack(self, g, m, v, sched: Optional[torch.Tensor] = None, neg_step_actor: float = 0.0,
                  neg_step_critic: float = 0.0, bc2_sqrt: float = 1.0,
                  one_minus_beta1: float = 0.1, beta2: float = 0.999,
                  one_minus_beta2: float = 0.001, eps: float = 1e-8,
                  next_rows: Optional[torch.Tensor] = None) -> None:
        """ppo_adam on the bound parameters (ppo_adam_sched when sched is given) that also
        refreshes the fused kernels' bf16 weight images; with next_rows, also gathers the next
        minibatch's rows from the staged records (ppo_adam_pack_gather)."""
        for name, t in (("g", g), ("m", m), ("v", v)):
            _need(t, name, torch.float32, (self.n_params,), self.device)
        if sched is not None:
            _need(sched, "sched", torch.float32, None, self.device)
            if sched.numel() < 3:
                raise RuntimeError("sched must hold 3 floats")
        if next_rows is not None:
            _need(next_rows, "next_rows", torch.int32, device=self.device)
            check(self.lib.ppo_adam_pack_gather(
                self._ctx, ptr(g), ptr(m), ptr(v), ptr(sched), neg_step_actor, neg_step_critic,
                bc2_sqrt, one_minus_beta1, beta2, one_minus_beta2, eps, ptr(next_rows),
                next_rows.numel(), _stream(self.device)))
            return
        check(self.lib.ppo_adam_pack(self._ctx, ptr(g), ptr(m), ptr(v), ptr(sched),
                                     neg_step_actor, neg_step_critic, bc2_sqrt, one_minus_beta1,
                                     beta2, one_minus_beta2, eps, _stream(self.device)))


# ==============================================================================================
# Context-free kernels
# ==============================================================================================
def _gae_check(value, next_value, reward, terminated, adv, vtarget, done) -> None:
    t, n = value.shape[0], value.shape[1]
    dev = value.device
    _need(value, "value", torch.float32, (t, n))
    _need(next_value, "next_value", torch.float32, (t, n), dev)
    if reward.dtype not in (torch.float32, torch.float64):
        raise ValueError("reward must be f32 or f64")
    _need(reward, "reward", None, (t, n), dev)
    _need(terminated, "terminated", None, (t, n), dev)
    if terminated.dtype not in (torch.bool, torch.uint8):
        raise ValueError("terminated must be bool/uint8")
    if done is not None:
        _need(done, "done", None, (t, n), dev)
    _need(adv, "adv", torch.float32, (t, n), dev)
    _need(vtarget, "vtarget", torch.float32, (t, n), dev)


def gae(value, next_value, reward, terminated, gamma: float, lmbda: float, adv, vtarget,
        done=None, force_last_done: bool = True) -> None:
    """A7/A8 on time-major (T, N) arrays (torchrl GAE semantics, f64 carry)."""
    lib = _lib.load()
    t, n = value.shape[0], value.shape[1]
    dev = value.device
    _gae_check(value, next_value, reward, terminated, adv, vtarget, done)
    check(lib.ppo_gae(ptr(value), ptr(next_value), ptr(reward), int(reward.dtype == torch.float64),
                      ptr(done), ptr(terminated), int(force_last_done), n, t, float(gamma),
                      float(lmbda), ptr(adv), ptr(vtarget), _stream(dev)))


def normalize_rows(x: torch.Tensor, scale: float = 1.0) -> None:
    """A6/A9: per-env (column of a time-major (T, N) array) standardisation over T, in place."""
    lib = _lib.load()
    if x.dtype not in (torch.float32, torch.float64):
        raise ValueError("x must be f32 or f64")
    _need(x, "x")
    t, n = x.shape[0], x.shape[1]
    check(lib.ppo_normalize_rows(ptr(x), int(x.dtype == torch.float64), n, t, float(scale),
                                 _stream(x.device)))


def obs_window_push(window: torch.Tensor, obs: torch.Tensor, reset: Optional[torch.Tensor] = None,
                    all_reset: bool = False) -> None:
    lib = _lib.load()
    n, o, w = window.shape
    _need(window, "window", torch.float64)
    if obs.dtype not in (torch.float32, torch.float64):
        raise ValueError("obs must be f32 or f64")
    _need(obs, "obs", None, (n, o), window.device)
    if reset is not None:
        _need(reset, "reset", None, (n,), window.device)
    check(lib.ppo_obs_window_push(ptr(window), ptr(obs), int(obs.dtype == torch.float64),
                                  ptr(reset), int(all_reset), n, o, w, _stream(window.device)))


def obs_normalize(window: torch.Tensor, state: torch.Tensor, normalize: bool = True) -> None:
    lib = _lib.load()
    n, o, w = window.shape
    _need(window, "window", torch.float64)
    _need(state, "state", torch.float32, device=window.device)
    if state.numel() != n * w * o:
        raise RuntimeError(f"state must hold (N, W, O) = {(n, w, o)} floats")
    edges = slice_edges(o)
    arr = (ctypes.c_int32 * len(edges))(*edges)
    check(lib.ppo_obs_normalize(ptr(window), ptr(state), n, o, w, arr, len(edges) - 1,
                                int(normalize), _stream(window.device)))


def perm_to_rows(perm: torch.Tensor, start: int, b: int, n_envs: int, horizon: int,
                 rows: torch.Tensor, shard: Optional[tuple] = None,
                 count: Optional[torch.Tensor] = None) -> None:
    lib = _lib.load()
    _need(perm, "perm", torch.int64)
    _need(rows, "rows", torch.int32, device=perm.device)
    lo, hi = shard if shard is not None else (0, 0)
    check(lib.ppo_perm_to_rows(ptr(perm), int(start), int(b), n_envs, horizon, lo, hi, ptr(rows),
                               ptr(count), _stream(perm.device)))


def feistel_rows(seed: int, epoch: int, start: int, b: int, n_envs: int, horizon: int,
                 rows: torch.Tensor) -> None:
    lib = _lib.load()
    _need(rows, "rows", torch.int32)
    check(lib.ppo_feistel_rows(seed, epoch, int(start), int(b), n_envs, horizon, ptr(rows),
                               _stream(rows.device)))


def adam(p, g, m, v, n_actor: int, neg_step_actor: float, neg_step_critic: float,
         one_minus_beta1: float, beta2: float, one_minus_beta2: float, bc2_sqrt: float,
         eps: float) -> None:
    lib = _lib.load()
    n = p.numel()
    for name, t in (("p", p), ("g", g), ("m", m), ("v", v)):
        _need(t, name, torch.float32, (n,), p.device)
    check(lib.ppo_adam(ptr(p), ptr(g), ptr(m), ptr(v), n, int(n_actor), neg_step_actor,
                       neg_step_critic, one_minus_beta1, beta2, one_minus_beta2, bc2_sqrt, eps,
                       _stream(p.device)))


def synthetic_env_step(base_obs, base_reward, base_term, action, obs_out, reward_out,
                       term_out) -> None:
    lib = _lib.load()
    n, o = base_obs.shape
    a = action.shape[1]
    dev = base_obs.device
    _need(base_obs, "base_obs", torch.float32)
    _need(base_reward, "base_reward", torch.float32, (n,), dev)
    _need(base_term, "base_term", None, (n,), dev)
    _need(action, "action", torch.float32, (n, a), dev)
    _need(obs_out, "obs_out", torch.float64, (n, o), dev)
    _need(reward_out, "reward_out", torch.float64, (n,), dev)
    _need(term_out, "term_out", None, (n,), dev)
    check(lib.ppo_synthetic_env_step(ptr(base_obs), ptr(base_reward), ptr(base_term), ptr(action),
                                     n, o, a, ptr(obs_out), ptr(reward_out), ptr(term_out),
                                     _stream(dev)))


def synthetic_test_step(base_obs, base_reward, base_term, action, window, step, reward_sum,
                        term_out) -> None:
    """One step of the evaluation env (ppo_synthetic_test_step): env 0 of the synthetic streams,
    window (O, W) f64 updated in place, the device step counter / reward sum / terminated flag
    advanced without a host synchronisation."""
    lib = _lib.load()
    t1, n, o = base_obs.shape
    dev = base_obs.device
    _need(base_obs, "base_obs", torch.float32)
    _need(base_reward, "base_reward", torch.float32, (t1 - 1, n), dev)
    _need(base_term, "base_term", None, (t1 - 1, n), dev)
    _need(action, "action", torch.float32, device=dev)
    _need(window, "window", torch.float64, device=dev)
    if window.numel() % o or window.shape[-2] != o:
        raise RuntimeError(f"window has shape {tuple(window.shape)}, expected (..., O={o}, W)")
    _need(step, "step", torch.int32, (1,), dev)
    _need(reward_sum, "reward_sum", torch.float64, (1,), dev)
    _need(term_out, "term_out", None, (1,), dev)
    check(lib.ppo_synthetic_test_step(ptr(base_obs), ptr(base_reward), ptr(base_term), t1 - 1, n,
                                      ptr(action), o, action.numel(), window.shape[-1],
                                      ptr(window), ptr(step), ptr(reward_sum), ptr(term_out),
                                      _stream(dev)))


def philox_normal(seed: int, offset: int, out: torch.Tensor,
                  counter: Optional[torch.Tensor] = None) -> None:
    """out[i] = the Philox normal at index offset (+ *counter, read on the device) + i: the draws
    of ppo_policy_step / ppo_observe_act in perf mode, bitwise."""
    lib = _lib.load()
    _need(out, "out", torch.float32)
    if counter is None:
        check(lib.ppo_philox_normal(seed, offset, ptr(out), out.numel(), _stream(out.device)))
        return
    _need(counter, "counter", torch.int64, (1,), out.device)
    check(lib.ppo_philox_normal_ctr(seed, offset, ptr(counter), ptr(out), out.numel(),
                                    _stream(out.device)))


def adam_sched(p, g, m, v, n_actor: int, sched: torch.Tensor, one_minus_beta1: float, beta2: float,
               one_minus_beta2: float, eps: float) -> None:
    """ppo_adam_sched: Adam with (neg_step_actor, neg_step_critic, bc2_sqrt) = sched[0:3] read
    from device memory at run time (graph-captured optimizer loops)."""
    lib = _lib.load()
    n = p.numel()
    for name, t in (("p", p), ("g", g), ("m", m), ("v", v)):
        _need(t, name, torch.float32, (n,), p.device)
    _need(sched, "sched", torch.float32, None, p.device)
    if sched.numel() < 3:
        raise RuntimeError("sched must hold 3 floats")
    check(lib.ppo_adam_sched(ptr(p), ptr(g), ptr(m), ptr(v), n, int(n_actor), ptr(sched),
                             one_minus_beta1, beta2, one_minus_beta2, eps, _stream(p.device)))
