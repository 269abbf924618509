"""CPU: the ENGINE's checkpoint files load into the REFERENCE's own modules and optimizers
(agent.py:47-72, features.py:134-165).

tests/golden/engine_ckpt/ was written on the GPU box by PPOEngineAgent.save() after one PPO
iteration on the engine (tools/make_engine_ckpt.py; actor 2x64, critic the reference's [128, 128],
W=1).  Here, where /root/reference exists (skipped elsewhere), the files are loaded with
weights_only=True into models.linear.actor.Actor / models.critic.Critic and torch.optim.Adam,
and must reproduce the engine's recorded forward (rtol 1e-5: HIP vs CPU summation order) and its
next Adam step (<= 2 ulp); the engine's configurations.json must restore through the reference's
positional Run.get_configurations.
"""
import os
import sys

import numpy as np
import pytest
import torch

REF_SRC = "/root/reference/src"
FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "engine_ckpt")

pytestmark = pytest.mark.skipif(not os.path.isdir(REF_SRC) or not os.path.isdir(FIXTURE),
                                reason="needs the reference sources and the engine fixture")


@pytest.fixture()
def reference():
    sys.path.insert(0, REF_SRC)
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from entities import features as F
    from gen_golden import _make_run
    from models.critic import Critic
    from models.linear.actor import Actor
    yield F, _make_run, Actor, Critic
    F.Run._instances.clear()


def test_reference_modules_load_engine_checkpoint(reference):
    F, make_ref_run, Actor, Critic = reference
    probe = np.load(os.path.join(FIXTURE, "probe.npz"))
    path = os.path.join(FIXTURE, "networks", str(int(probe["episode"])))
    make_ref_run(17, 1, 6, [64, 64], "ReLU")
    nets = torch.nn.ModuleDict()
    nets["actor"] = Actor()
    nets["critic"] = Critic()
    nets.load_state_dict(torch.load(f"{path}/networks.pth", weights_only=True))  # strict keys
    x = torch.from_numpy(probe["x"])
    with torch.no_grad():
        mean, std = nets["actor"](x)
        value = nets["critic"](x)[:, 0, :]
    torch.testing.assert_close(mean, torch.from_numpy(probe["mean"]), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(value, torch.from_numpy(probe["value"]), rtol=1e-5, atol=1e-6)
    assert torch.equal(std, torch.from_numpy(probe["std"]))
    opts = {k: torch.optim.Adam(nets[k].parameters(), lr=1.0) for k in ("actor", "critic")}
    for k, o in opts.items():
        o.load_state_dict(torch.load(f"{path}/optimizer_{k}.pth", weights_only=True))
    assert opts["actor"].param_groups[0]["lr"] < 1.0  # the engine's (decayed) lr was restored
    grad = torch.from_numpy(probe["grad"])
    off = 0
    for p in nets.parameters():
        p.grad = grad[off:off + p.numel()].view(p.shape).clone()
        off += p.numel()
    opts["critic"].step()
    opts["actor"].step()
    got = torch.cat([p.detach().flatten() for p in nets.parameters()])
    exp = torch.from_numpy(probe["params_after"])
    ulp = torch.finfo(torch.float32).eps * exp.abs().clamp_min(1e-30)
    assert bool(((got - exp).abs() <= 2 * ulp).all()), float(((got - exp).abs() / ulp).max())


def test_reference_restores_engine_configurations(reference):
    F, *_ = reference
    F.Run._instances.clear()
    run = F.Run.get_configurations(FIXTURE)  # positional restore (features.py:145-165)
    assert run.network_config.input_shape == 17
    assert run.network_config.linear_hidden_shapes == [64, 64]
    assert run.network_config.activation_class is torch.nn.ReLU
    assert run.dtype is torch.float32


def test_reference_lstm_modules_load_engine_state_dict(tmp_path):
    """The LSTM agent's networks (lstm.EngineLSTMActor / EngineLSTMCritic, the state_dict that
    LSTMEngineAgent.save writes to networks.pth) load strictly into the reference's own
    LSTMActor / LSTMCritic (weights_only), and the reference forward on those parameters equals
    the oracle's restated BiLSTM forward."""
    sys.path.insert(0, REF_SRC)
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from entities import features as F
    from gen_golden_lstm import _make_run
    from models.lstm.lstm_actor import LSTMActor
    from models.lstm.lstm_critic import LSTMCritic
    from mujoco_reinforcement_learning_amd.lstm import EngineLSTMActor, EngineLSTMCritic
    from oracle import lstm_ref as L
    from oracle.ppo_ref import RefConfig
    try:
        obs, window, act, latent, hidden = 17, 3, 6, 8, [16, 16]
        torch.manual_seed(5)
        nets = torch.nn.ModuleDict()
        nets["actor"] = EngineLSTMActor(obs, latent, 1, window, hidden, act, torch.nn.ReLU, True,
                                        0.01)
        nets["critic"] = EngineLSTMCritic(obs, latent, hidden, torch.nn.ReLU, True, 0.01)
        torch.save({k: v.detach().cpu() for k, v in nets.state_dict().items()},
                   tmp_path / "networks.pth")
        _make_run(obs, window, act, latent, 1, hidden, "ReLU")
        ref = torch.nn.ModuleDict()
        ref["actor"] = LSTMActor()
        ref["critic"] = LSTMCritic()
        ref.load_state_dict(torch.load(tmp_path / "networks.pth", weights_only=True))  # strict
        cfg = RefConfig(obs_dim=obs, act_dim=act, window=window, actor_hidden=tuple(hidden),
                        critic_hidden=tuple(hidden))
        oracle = L.RefLSTMAgent(cfg, latent, 1)
        oracle.networks.load_state_dict(torch.load(tmp_path / "networks.pth", weights_only=True))
        x = torch.randn(9, window, obs, generator=torch.Generator().manual_seed(3))
        with torch.no_grad():
            mean, std_rep = ref["actor"](x)
            value = ref["critic"](x)
            m2, s2 = oracle.networks["actor"](x)
            v2 = oracle.networks["critic"](x)
        torch.testing.assert_close(mean, m2, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(std_rep[0], s2, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(value, v2, rtol=1e-6, atol=1e-7)
    finally:
        F.Run._instances.clear()
