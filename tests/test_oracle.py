"""CPU: pin the oracle (oracle/ppo_ref.py) against the reference's own modules and known answers.

* MLP init + forward: bit-exact against tests/golden/reference_mlp.npz, which
  tests/golden/gen_golden.py produced by importing /root/reference/src/models.
* GAE (torchrl 0.6.0, absent here): hand-derived known answers + the f64-carry dtype walk.
  Parity against the real torchrl is unpinned (no reference test or fixture covers it).
* RNG contract: Normal.sample == randn*std + mean, same generator consumption.
"""
import hashlib
import os

import numpy as np
import pytest
import torch

from oracle.ppo_ref import (RefAgent, RefConfig, RefSyntheticEnv, SHAPE_ERR, calculate_advantages,
                            generalized_advantage_estimate, get_state, normalize_state, rollout,
                            train)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_mlp.npz")


def _golden_cases():
    return sorted({k.split("/")[0] for k in np.load(GOLDEN).files})


def _cfg_from_meta(z, name):
    seed, obs, window, a, n_a, n_c, *widths = (int(v) for v in z[f"{name}/meta"])
    return seed, RefConfig(obs_dim=obs, window=window, act_dim=a,
                           actor_hidden=tuple(widths[:n_a]),
                           critic_hidden=tuple(widths[n_a:n_a + n_c]),
                           activation=str(z[f"{name}/activation"]))


def _check_state_dict(sd, z, name):
    """Every tensor equals the reference's: the stored array when the fixture keeps it (small
    nets), else the sha256 of its bytes."""
    keys = sorted(k[len(name) + len("/sha256/"):] for k in z.files
                  if k.startswith(f"{name}/sha256/"))
    assert sorted(sd.keys()) == keys
    for k, v in sd.items():
        arr = v.detach().contiguous().numpy()
        if f"{name}/{k}" in z.files:
            assert np.array_equal(arr, z[f"{name}/{k}"]), k
        assert hashlib.sha256(arr.tobytes()).hexdigest() == str(z[f"{name}/sha256/{k}"]), k


def test_golden_covers_the_baseline_and_main_py_nets():
    names = _golden_cases()
    assert {"humanoid_relu_3x512", "main_py_net", "ant_relu_2x256", "relu_2x256"} <= set(names)


@pytest.mark.parametrize("name", _golden_cases())
def test_oracle_models_match_reference_golden(name):
    z = np.load(GOLDEN)
    seed, cfg = _cfg_from_meta(z, name)
    torch.manual_seed(seed)
    agent = RefAgent(cfg)
    _check_state_dict(agent.networks.state_dict(), z, name)
    x = torch.from_numpy(z[f"{name}/x"])
    with torch.no_grad():
        mean, std = agent.networks["actor"](x)
        value = agent.networks["critic"](x)
    assert np.array_equal(mean.numpy(), z[f"{name}/mean"])
    assert np.array_equal(std.numpy(), z[f"{name}/std"])
    assert np.array_equal(value.numpy(), z[f"{name}/value"])


@pytest.mark.parametrize("name", _golden_cases())
def test_engine_model_init_matches_reference_golden(name):
    """The product's CPU-side init (models._Block + EngineActor/EngineCritic) replays the
    reference RNG order: same seed -> the reference's exact parameters and state_dict keys."""
    from mujoco_reinforcement_learning_amd.models import EngineActor, EngineCritic
    z = np.load(GOLDEN)
    seed, cfg = _cfg_from_meta(z, name)
    acts = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh, "elu": torch.nn.ELU}
    torch.manual_seed(seed)
    nets = torch.nn.ModuleDict()
    nets["actor"] = EngineActor(cfg.obs_dim * cfg.window, cfg.actor_hidden, cfg.act_dim,
                                acts[cfg.activation], True, 1.0)
    nets["critic"] = EngineCritic(cfg.obs_dim * cfg.window, cfg.critic_hidden,
                                  acts[cfg.activation])
    _check_state_dict(nets.state_dict(), z, name)


def test_gae_known_answer_mid_termination():
    # gamma = lambda = 0.5, T = 3, termination at t = 1 (hand-derived):
    # delta = [1 + .5*2 - 1, 1 + 0 - 2, 1 + .5*4 - 3] = [1, -1, 0]; disc = .25*[1, 0, 0]
    # A2 = 0, A1 = -1, A0 = 1 + .25*(-1) = .75;  vtarget = A + V = [1.75, 1, 3]
    v = torch.tensor([[[1.0], [2.0], [3.0]]])
    vn = torch.tensor([[[2.0], [3.0], [4.0]]])
    r = torch.tensor([[[1.0], [1.0], [1.0]]], dtype=torch.float64)
    term = torch.tensor([[[False], [True], [False]]])
    done = term.clone()
    done[:, -1] = True
    adv, vt = generalized_advantage_estimate(0.5, 0.5, v, vn, r, done, term)
    assert adv.dtype == torch.float32
    assert adv.flatten().tolist() == [0.75, -1.0, 0.0]
    assert vt.flatten().tolist() == [1.75, 1.0, 3.0]


def test_gae_known_answer_zero_discount_and_zero_rewards():
    g = torch.Generator().manual_seed(3)
    v = torch.randn(4, 5, 1, generator=g)
    vn = torch.randn(4, 5, 1, generator=g)
    r = torch.randn(4, 5, 1, generator=g, dtype=torch.float64)
    term = torch.zeros(4, 5, 1, dtype=torch.bool)
    adv, _ = generalized_advantage_estimate(0.0, 0.0, v, vn, r, term.clone(), term)
    assert torch.equal(adv, (r - v.double()).float())
    z = torch.zeros(2, 6, 1)
    t0 = torch.zeros(2, 6, 1, dtype=torch.bool)
    adv, vt = generalized_advantage_estimate(0.99, 0.98, z, z, z.double(), t0 | True, t0)
    assert torch.count_nonzero(adv) == 0 and torch.count_nonzero(vt) == 0


def test_gae_carries_in_f64():
    """prev_advantage is the f64 RHS of the chained assignment: equal to an explicit python-float
    loop, and different from an all-f32 recurrence somewhere on a long horizon."""
    g = torch.Generator().manual_seed(0)
    n, t = 64, 128
    v = torch.randn(n, t, 1, generator=g)
    vn = torch.randn(n, t, 1, generator=g)
    r = torch.randn(n, t, 1, generator=g, dtype=torch.float64)
    term = torch.rand(n, t, 1, generator=g) < 0.02
    done = term.clone()
    done[:, -1] = True
    adv, _ = generalized_advantage_estimate(0.99, 0.98, v, vn, r, done, term)
    gf, lg = np.float32(0.99), np.float32(0.98 * 0.99)
    ref = np.empty((n, t), np.float32)
    f32 = np.empty((n, t), np.float32)
    for i in range(n):
        prev, prevf = 0.0, np.float32(0)
        for k in reversed(range(t)):
            gnt = gf * np.float32(0.0 if term[i, k, 0] else 1.0)
            gv = np.float32(gnt * np.float32(vn[i, k, 0]))
            delta = (float(r[i, k, 0]) + float(gv)) - float(v[i, k, 0])
            disc = np.float32(lg * np.float32(0.0 if done[i, k, 0] else 1.0))
            prev = delta + prev * float(disc)
            ref[i, k] = np.float32(prev)
            prevf = np.float32(np.float32(delta) + prevf * disc)
            f32[i, k] = prevf
    assert np.array_equal(adv[..., 0].numpy(), ref)
    assert not np.array_equal(ref, f32)


def test_gae_shape_error():
    z = torch.zeros(2, 3, 1)
    with pytest.raises(RuntimeError, match="unique shape"):
        generalized_advantage_estimate(0.99, 0.98, z, z, torch.zeros(2, 3), z.bool(), z.bool())
    assert "unique shape" in SHAPE_ERR


def test_normal_sample_rng_contract():
    """Normal(mean,std).sample() == randn(shape)*std + mean bitwise with identical generator
    consumption (what lets the engine's parity mode draw eps on the host)."""
    mean = torch.randn(37, 6)
    std = torch.rand(6).exp()[None].repeat(37, 1)
    torch.manual_seed(5)
    a = torch.distributions.Normal(mean, std).sample()
    after_a = torch.rand(4)
    torch.manual_seed(5)
    b = torch.randn(37, 6) * std + mean
    after_b = torch.rand(4)
    assert torch.equal(a, b) and torch.equal(after_a, after_b)


def test_obs_normalisation_slices():
    g = torch.Generator().manual_seed(1)
    w = torch.randn(5, 17, 3, generator=g, dtype=torch.float64)
    w[0, :, 1] = 2.5  # constant slot -> std 0 -> divided by 1
    out = normalize_state(w.clone())
    x = w[1, :, 0]
    assert torch.allclose(out[1, :, 0], (x - x.mean()) / x.std())
    assert torch.equal(out[0, :, 1], torch.zeros(17, dtype=torch.float64))
    # O=23: slice [22:23] holds one feature -> torch.std gives NaN (reference behaviour)
    w2 = torch.randn(2, 23, 1, generator=g, dtype=torch.float64)
    out2 = normalize_state(w2.clone())
    assert torch.isnan(out2[:, 22]).all() and torch.isfinite(out2[:, :22]).all()
    st = get_state(w, True)
    assert st.shape == (5, 3, 17) and st.dtype == torch.float32


def _small_iteration(seed=0, n=8, t=16, b=32, epochs=2):
    cfg = RefConfig(num_envs=n, horizon=t, batch_size=b, epochs=epochs)
    g = torch.Generator().manual_seed(100 + seed)
    env = RefSyntheticEnv(torch.randn(t + 1, n, 17, generator=g),
                          torch.rand(t, n, generator=g) * 2 - 1,
                          torch.rand(t, n, generator=g) < 0.05, 1, 6)
    torch.manual_seed(seed)
    agent = RefAgent(cfg)
    mem = rollout(env, agent)
    calculate_advantages(mem, cfg)
    return cfg, agent, mem


def test_oracle_rollout_shapes_and_dtypes():
    cfg, agent, mem = _small_iteration()
    n, t = cfg.num_envs, cfg.horizon
    assert mem["current_state"].shape == (n, t, 1, 17)
    assert mem["reward"].dtype == torch.float64 and mem["reward"].shape == (n, t, 1)
    assert mem["advantage"].shape == (n, t, 1)
    # V'_t == V_{t+1} exactly (same critic on the same tensor)
    assert torch.equal(mem["next_state_value"][:, :-1], mem["current_state_value"][:, 1:])


def test_oracle_train_changes_params_and_is_deterministic():
    cfg, agent, mem = _small_iteration()
    before = torch.cat([p.detach().flatten().clone() for p in agent.networks.parameters()])
    torch.manual_seed(11)
    la, lc = train(agent, mem)
    after = torch.cat([p.detach().flatten() for p in agent.networks.parameters()])
    assert np.isfinite(la) and np.isfinite(lc)
    assert not torch.equal(before, after)
    cfg2, agent2, mem2 = _small_iteration()
    torch.manual_seed(11)
    train(agent2, mem2)
    after2 = torch.cat([p.detach().flatten() for p in agent2.networks.parameters()])
    assert torch.equal(after, after2)


def test_oracle_train_empty_epoch_raises_like_reference():
    cfg, agent, mem = _small_iteration()
    agent.cfg.batch_size = cfg.num_envs * cfg.horizon + 1  # int(T*N/B) == 0 batches
    with pytest.raises(ZeroDivisionError):
        train(agent, mem)
