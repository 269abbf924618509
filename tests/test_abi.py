"""CPU: the C-ABI library builds, loads, exports every symbol include/ppo_engine.h declares, and
rejects bad arguments with the documented error codes (no GPU needed: argument checks run before
any HIP call)."""
import ctypes
import os
import re
import subprocess

import pytest

from mujoco_reinforcement_learning_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ppo_engine.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char \*)\s*\*?(ppo_\w+)\(", text,
                                 re.M)))


def test_header_declares_the_bound_symbols():
    declared = _declared()
    assert len(declared) >= 16
    assert sorted(_lib.EXPORTED_SYMBOLS) == declared


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (ppo_\w+)", out))
    for name in _declared():
        assert name in exported, name
        assert getattr(lib, name) is not None
    assert lib.ppo_abi_version() == 1


def test_bad_arguments_return_einval_with_message():
    lib = _lib.load()
    rc = lib.ppo_gae(None, None, None, 0, None, None, 1, 4, 4, 0.99, 0.98, None, None, None)
    assert rc == -22
    assert b"null" in lib.ppo_last_error()
    rc = lib.ppo_adam(None, None, None, None, 10, 0, 0.0, 0.0, 0.1, 0.999, 0.001, 1.0, 1e-8, None)
    assert rc == -22
    cfg = _lib.NetCfg()
    cfg.obs_dim, cfg.window, cfg.act_dim = 17, 1, 0
    handle = ctypes.c_void_p()
    assert lib.ppo_ctx_create(ctypes.byref(cfg), 0, ctypes.byref(handle)) == -22
    assert b"act_dim" in lib.ppo_last_error()
    with pytest.raises(_lib.EngineError, match="act_dim"):
        _lib.check(-22)


def test_comm_entry_points_resolve_rccl_and_check_arguments():
    """The data-parallel exchange (comm.hip, SURVEY.md s8(b) ppo_allreduce_grads): RCCL resolves
    at run time (the instance torch loaded, else ROCm's), a unique id can be drawn without a GPU,
    and bad arguments fail with EINVAL before any collective."""
    lib = _lib.load()
    assert lib.ppo_comm_version() >= 22000  # NCCL_VERSION_CODE 2.20+
    uid = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    assert lib.ppo_comm_unique_id(uid) == 0
    assert any(bytes(uid))
    handle = ctypes.c_void_p()
    assert lib.ppo_comm_create(uid, 2, 2, 0, ctypes.byref(handle)) == -22
    assert b"rank 2 of 2" in lib.ppo_last_error()
    assert lib.ppo_allreduce_grads(None, None, 4, None) == -22
    assert lib.ppo_comm_allreduce(None, None, 4, None) == -22
    assert lib.ppo_ctx_loss_entropy_share(None, 0.0) == -22
