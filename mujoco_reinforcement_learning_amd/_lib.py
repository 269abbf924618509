"""ctypes binding of libppo_engine.so (the C-ABI declared in include/ppo_engine.h).

The product path has exactly one implementation: the gfx950 HIP kernels in this library.  If the
library is missing or cannot be loaded this module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_int64, c_uint64, c_void_p

LIB_NAME = "libppo_engine.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

PPO_MAX_LAYERS = 8
ACT_CODES = {"relu": 0, "tanh": 1, "elu": 2}
PREC_CODES = {"f32": 0, "bf16": 1}  # PPO_PREC_* (include/ppo_engine.h)


class NetCfg(ctypes.Structure):
    """``ppo_net_cfg`` (include/ppo_engine.h)."""
    _fields_ = [
        ("obs_dim", c_int32),
        ("window", c_int32),
        ("act_dim", c_int32),
        ("activation", c_int32),
        ("actor_use_bias", c_int32),
        ("n_actor_hidden", c_int32),
        ("actor_hidden", c_int32 * PPO_MAX_LAYERS),
        ("n_critic_hidden", c_int32),
        ("critic_hidden", c_int32 * PPO_MAX_LAYERS),
        ("output_max_value", c_float),
        ("max_rows", c_int32),
    ]


class LstmCfg(ctypes.Structure):
    """``ppo_lstm_cfg`` (include/ppo_engine.h)."""
    _fields_ = [
        ("obs_dim", c_int32),
        ("window", c_int32),
        ("act_dim", c_int32),
        ("activation", c_int32),
        ("use_bias", c_int32),
        ("latent", c_int32),
        ("actor_layers", c_int32),
        ("n_hidden", c_int32),
        ("hidden", c_int32 * PPO_MAX_LAYERS),
        ("max_rows", c_int32),
    ]


class CnnCfg(ctypes.Structure):
    """``ppo_cnn_cfg`` (include/ppo_engine.h)."""
    _fields_ = [
        ("height", c_int32),
        ("width", c_int32),
        ("channels", c_int32),
        ("act_dim", c_int32),
        ("activation", c_int32),
        ("use_bias", c_int32),
        ("n_hidden", c_int32),
        ("hidden", c_int32 * PPO_MAX_LAYERS),
        ("output_max_value", c_float),
        ("max_rows", c_int32),
    ]


PPO_MAX_GROUPS = 4


class HostPoolDesc(ctypes.Structure):
    """``ppo_host_pool_desc`` (include/ppo_engine.h)."""
    _fields_ = [
        ("groups", c_int32),
        ("group_lo", c_int32 * PPO_MAX_GROUPS),
        ("group_hi", c_int32 * PPO_MAX_GROUPS),
        ("worker_lo", c_int32 * PPO_MAX_GROUPS),
        ("worker_hi", c_int32 * PPO_MAX_GROUPS),
        ("gen", c_int64 * PPO_MAX_GROUPS),
        ("ctrl", c_void_p),
        ("done", c_void_p),
        ("action", c_void_p),
        ("obs", c_void_p),
        ("reward", c_void_p),
        ("term", c_void_p),
        ("action_dev", c_void_p),
        ("obs_dev", c_void_p),
        ("reward_dev", c_void_p),
        ("term_dev", c_void_p),
    ]


_SIGNATURES = {
    "ppo_abi_version": (c_int, []),
    "ppo_last_error": (ctypes.c_char_p, []),
    "ppo_ctx_create": (c_int, [POINTER(NetCfg), c_int, POINTER(c_void_p)]),
    "ppo_ctx_destroy": (c_int, [c_void_p]),
    "ppo_param_count": (c_int64, [c_void_p, c_int]),
    "ppo_bind_params": (c_int, [c_void_p, c_void_p]),
    "ppo_param_offsets": (c_int, [c_void_p, POINTER(c_int64), c_int]),
    "ppo_obs_window_push": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                                    c_int, c_void_p]),
    "ppo_obs_normalize": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, POINTER(c_int32), c_int,
                                  c_int, c_void_p]),
    "ppo_policy_step": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint64, c_uint64, c_void_p,
                                c_void_p, c_void_p, c_void_p, c_void_p]),
    "ppo_normalize_rows": (c_int, [c_void_p, c_int, c_int, c_int, c_double, c_void_p]),
    "ppo_gae": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int,
                        c_int, c_double, c_double, c_void_p, c_void_p, c_void_p]),
    "ppo_perm_to_rows": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                 c_void_p, c_void_p]),
    "ppo_feistel_rows": (c_int, [c_uint64, c_uint64, c_int64, c_int, c_int, c_int, c_void_p,
                                 c_void_p]),
    "ppo_minibatch_grad": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_int, c_void_p, c_float, c_float, c_float, c_float,
                                   c_float, c_void_p, c_void_p, c_void_p]),
    "ppo_adam": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_float,
                         c_float, c_float, c_float, c_float, c_float, c_float, c_void_p]),
    "ppo_synthetic_env_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                       c_void_p, c_void_p, c_void_p, c_void_p]),
    "ppo_philox_normal": (c_int, [c_uint64, c_uint64, c_void_p, c_int64, c_void_p]),
    "ppo_philox_normal_ctr": (c_int, [c_uint64, c_uint64, c_void_p, c_void_p, c_int64, c_void_p]),
    "ppo_synthetic_test_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                        c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p]),
    "ppo_ctx_set_rng_counter": (c_int, [c_void_p, c_void_p]),
    "ppo_ctx_fused_direct": (c_int, [c_void_p, c_int]),
    "ppo_ctx_set_precision": (c_int, [c_void_p, c_int]),
    "ppo_ctx_timing": (c_int, [c_void_p, c_int, c_int]),
    "ppo_ctx_timing_read": (c_int, [c_void_p, c_int, POINTER(c_double), POINTER(c_int64),
                                    POINTER(c_double), POINTER(c_double)]),
    "ppo_kernel_class_name": (ctypes.c_char_p, [c_int]),
    "ppo_ctx_timing_kernel": (c_int, [c_void_p, c_int, POINTER(ctypes.c_char_p), POINTER(c_int),
                                      POINTER(c_double), POINTER(c_int64), POINTER(c_double),
                                      POINTER(c_double)]),
    "ppo_ctx_phase_stamps": (c_int, [c_void_p, c_int, c_void_p, c_int]),
    "ppo_pack_weights": (c_int, [c_void_p, c_void_p]),
    "ppo_adam_sched": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                               ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                               c_void_p]),
    "ppo_observe_act": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                                c_int, c_void_p, c_int, c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ppo_ctx_fused_active": (c_int, [c_void_p]),
    "ppo_host_register": (c_int, [c_void_p, c_int64]),
    "ppo_host_unregister": (c_int, [c_void_p]),
    "ppo_memcpy_async": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "ppo_host_device_ptr": (c_int, [c_void_p, POINTER(c_void_p)]),
    "ppo_stage_records": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_int64, c_void_p]),
    "ppo_gae_stage_records": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                      c_void_p, c_int, c_int, c_int, c_double, c_double, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ppo_minibatch_grad_staged": (c_int, [c_void_p, c_void_p, c_int, c_void_p, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                          ctypes.c_float, c_void_p, c_void_p, c_int, c_void_p]),
    "ppo_update_step_staged": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int]
                               + [ctypes.c_float] * 5 + [c_void_p] * 5 + [ctypes.c_float] * 7
                               + [c_int, c_void_p]),
    "ppo_gather_staged_rows": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "ppo_adam_pack_gather": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
                             + [ctypes.c_float] * 7 + [c_void_p, c_int, c_void_p]),
    "ppo_adam_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float,
                              ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                              ctypes.c_float, ctypes.c_float, c_void_p]),
    "ppo_host_rollout": (c_int, [c_void_p, POINTER(HostPoolDesc), c_void_p, POINTER(c_int32), c_int,
                                 c_int] + [c_void_p] * 7 + [c_int] * 5 + [c_void_p, c_uint64,
                                                                       c_uint64, c_void_p]),
    # windowed BiLSTM actor-critic (bilstm.hip)
    "ppo_lstm_ctx_create": (c_int, [POINTER(LstmCfg), c_int, POINTER(c_void_p)]),
    "ppo_lstm_ctx_destroy": (c_int, [c_void_p]),
    "ppo_lstm_param_layout": (c_int, [c_void_p, POINTER(c_int64), c_int, POINTER(c_int64),
                                      POINTER(c_int64)]),
    "ppo_lstm_bind_params": (c_int, [c_void_p, c_void_p]),
    "ppo_lstm_set_precision": (c_int, [c_void_p, c_int]),
    "ppo_lstm_forward": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p]),
    "ppo_lstm_policy_step": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint64, c_uint64,
                                     c_void_p, c_void_p, c_void_p, c_void_p]),
    "ppo_lstm_minibatch_grad": (c_int, [c_void_p] + [c_void_p] * 6 + [c_int, c_void_p, c_void_p]
                                + [ctypes.c_float] * 5 + [c_void_p]),
    "ppo_lstm_fused_step": (c_int, [c_void_p, c_int]),
    "ppo_lstm_timing": (c_int, [c_void_p, c_int, c_int]),
    "ppo_lstm_timing_kernel": (c_int, [c_void_p, c_int, POINTER(ctypes.c_char_p), POINTER(c_int),
                                       POINTER(c_double), POINTER(c_int64), POINTER(c_double),
                                       POINTER(c_double)]),
    # pixel-observation actor-critic (cnn_engine.hip, conv.h)
    "ppo_cnn_ctx_create": (c_int, [POINTER(CnnCfg), c_int, POINTER(c_void_p)]),
    "ppo_cnn_ctx_destroy": (c_int, [c_void_p]),
    "ppo_cnn_param_layout": (c_int, [c_void_p, POINTER(c_int64), c_int, POINTER(c_int64),
                                     POINTER(c_int64)]),
    "ppo_cnn_bind_params": (c_int, [c_void_p, c_void_p]),
    "ppo_cnn_set_precision": (c_int, [c_void_p, c_int]),
    "ppo_cnn_set_rng_counter": (c_int, [c_void_p, c_void_p]),
    "ppo_cnn_forward": (c_int, [c_void_p, c_void_p, c_int] + [c_void_p] * 5),
    "ppo_cnn_policy_step": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint64, c_uint64]
                            + [c_void_p] * 5),
    "ppo_cnn_minibatch_grad": (c_int, [c_void_p] + [c_void_p] * 6 + [c_int, c_void_p, c_void_p]
                               + [ctypes.c_float] * 5 + [c_void_p]),
    "ppo_cnn_timing": (c_int, [c_void_p, c_int, c_int]),
    "ppo_cnn_timing_kernel": (c_int, [c_void_p, c_int, POINTER(ctypes.c_char_p), POINTER(c_int),
                                      POINTER(c_double), POINTER(c_int64), POINTER(c_double),
                                      POINTER(c_double)]),
    # wide layered path (wide_gemm.hip)
    "ppo_wide_gemm": (c_int, [c_int, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_int64,
                              c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_int,
                              c_void_p, c_void_p]),
    "ppo_synthetic_pixel_step": (c_int, [ctypes.c_uint32, c_int, c_void_p, c_int, c_int, c_int,
                                         c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p]),
    # data-parallel gradient exchange (comm.hip) and the logged loss's entropy share
    "ppo_comm_version": (c_int, []),
    "ppo_comm_unique_id": (c_int, [c_void_p]),
    "ppo_comm_create": (c_int, [c_void_p, c_int, c_int, c_int, POINTER(c_void_p)]),
    "ppo_comm_destroy": (c_int, [c_void_p]),
    "ppo_comm_allreduce": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "ppo_comm_check": (c_int, [c_void_p]),
    "ppo_comm_query": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "ppo_ctx_set_comm": (c_int, [c_void_p, c_void_p]),
    "ppo_allreduce_grads": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "ppo_ctx_loss_entropy_share": (c_int, [c_void_p, c_float]),
    "ppo_lstm_loss_entropy_share": (c_int, [c_void_p, c_float]),
    "ppo_cnn_loss_entropy_share": (c_int, [c_void_p, c_float]),
}

COMM_ID_BYTES = 128  # PPO_COMM_ID_BYTES

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib = None


class EngineError(RuntimeError):
    """A non-zero return code from the C-ABI (message from ``ppo_last_error``)."""


def load() -> ctypes.CDLL:
    """Load (once) and type the native library; raise if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP engine first (python -c 'import "
            "__graft_entry__ as g; g.build()' or make -C mujoco_reinforcement_learning_amd)")
    if os.environ.get("PPO_SEGV_MAPS") == "1":
        # diagnostics: a fatal SIGSEGV first dumps /proc/self/maps (csrc/host/crash_maps.c)
        ctypes.CDLL(os.path.join(os.path.dirname(LIB_PATH), "libppo_hostenv.so"))
    lib = ctypes.CDLL(LIB_PATH)
    for name, (restype, argtypes) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = restype
        fn.argtypes = argtypes
    if lib.ppo_abi_version() != 1:
        raise ImportError(f"{LIB_PATH}: ABI version {lib.ppo_abi_version()} != 1")
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().ppo_last_error().decode(errors="replace")
        raise EngineError(msg or f"ppo engine error {rc}")


def ptr(t) -> int:
    """Device pointer of a torch tensor (or 0 for None)."""
    if t is None:
        return None
    return t.data_ptr()
