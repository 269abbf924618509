"""GPU: one full PPO iteration (rollout -> GAE -> E epochs of minibatch updates) through the
drop-in classes, against the oracle on the same seeds and synthetic streams.

Bars: GAE on the engine's own rollout is bit-exact; rollout tensors and post-update parameters
agree within the tolerances printed in each assert (the f32 MLP sums in a different order from
CPU MKL, and Adam's early steps are ~lr*sign(g), so a near-zero gradient component can flip the
sign of a step -- bounded by 2*lr per step).
"""
import pytest
import torch

from oracle import ppo_ref as R

pytestmark = pytest.mark.gpu


def _setup(gpu, n=16, t=32, b=128, epochs=2, hidden=(64, 64), p_term=0.05, rng="torch", seed=0,
           **kw):
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    streams = make_synthetic_streams(n, t, 17, seed=seed + 5, p_terminate=p_term)
    run = make_run(num_envs=n, horizon=t, hidden=hidden, batch_size=b, epochs=epochs, rng=rng,
                   seed=seed, **kw)
    torch.manual_seed(seed)
    agent = PPOEngineAgent(run, device=gpu)
    helper = SyntheticVecEnvHelper(streams, run, device=gpu)
    algo = PPOEngine(helper, agent, log=lambda m: None)
    cfg = R.RefConfig(num_envs=n, horizon=t, actor_hidden=hidden, critic_hidden=hidden,
                      batch_size=b, epochs=epochs,
                      normalize_advantage=kw.get("normalize_advantage", False),
                      normalize_rewards=kw.get("normalize_rewards", False))
    torch.manual_seed(seed)
    ref = R.RefAgent(cfg)
    env = R.RefSyntheticEnv(streams["base_obs"], streams["base_reward"],
                            streams["base_terminated"], 1, 6)
    return algo, agent, ref, env, cfg


@pytest.mark.parametrize("kw", [{}, {"normalize_advantage": True, "normalize_rewards": True}])
def test_iteration_matches_oracle(gpu, kw):
    algo, agent, ref, env, cfg = _setup(gpu, **kw)
    assert torch.equal(agent.packed_params().cpu(), R.flat_params(ref))
    torch.manual_seed(1234)
    mem = algo.rollout()
    algo.calculate_advantages(mem)
    torch.manual_seed(1234)
    ref_mem = R.rollout(env, ref)
    R.calculate_advantages(ref_mem, cfg)

    # GAE of the engine's own rollout, recomputed by the oracle: bit-exact
    rewards = mem["reward"].cpu()
    if cfg.normalize_rewards:
        rewards = rewards - rewards.mean(dim=1).unsqueeze(1)
        rewards = rewards / rewards.std(dim=1).unsqueeze(1)
    term = mem["terminated"].cpu().unsqueeze(-1)
    done = term.clone()
    done[:, -1] = True
    adv_own, vt_own = R.generalized_advantage_estimate(
        0.99, 0.98, mem["current_state_value"].cpu(), mem["next_state_value"].cpu(), rewards,
        done, term)
    if not cfg.normalize_advantage:
        assert torch.equal(mem["advantage"].cpu(), adv_own)
        assert torch.equal(mem["current_state_value_target"].cpu(), vt_own)

    # rollout vs oracle rollout
    for key, tol in (("current_state", 1e-5), ("current_state_value", 1e-5),
                     ("next_state_value", 1e-5), ("action", 1e-5), ("action_log_prob", 1e-4),
                     ("reward", 1e-6), ("advantage", 1e-4), ("current_state_value_target", 1e-4)):
        a, r = mem[key].cpu(), ref_mem[key]
        assert a.shape == r.shape, key
        torch.testing.assert_close(a.to(r.dtype), r, rtol=tol, atol=tol, msg=key)
    assert torch.equal(mem["terminated"].cpu(), ref_mem["terminated"])

    # update: same RNG stream for randperm and the dropped ppo.py:110 samples
    torch.manual_seed(99)
    algo.train(mem)
    torch.manual_seed(99)
    R.train(ref, ref_mem, 0)
    p_eng, p_ref = agent.packed_params().cpu(), R.flat_params(ref)
    diff = (p_eng - p_ref).abs()
    n_steps = cfg.epochs * (cfg.num_envs * cfg.horizon // cfg.batch_size)
    lr = cfg.learning_rate
    assert float(diff.max()) <= 2 * lr * n_steps, float(diff.max())
    frac_tight = float((diff <= 1e-5 * p_ref.abs() + 1e-7).float().mean())
    assert frac_tight >= 0.95, frac_tight
    assert agent.optimizers["actor"].lr == ref.optimizers["actor"].param_groups[0]["lr"]


def test_single_minibatch_update_tight(gpu):
    """One minibatch (B = N*T, E = 1): post-Adam params within 1e-5 rtol except sign-flip steps."""
    algo, agent, ref, env, cfg = _setup(gpu, n=32, t=16, b=512, epochs=1)
    torch.manual_seed(7)
    mem = algo.rollout()
    algo.calculate_advantages(mem)
    torch.manual_seed(7)
    ref_mem = R.rollout(env, ref)
    R.calculate_advantages(ref_mem, cfg)
    torch.manual_seed(8)
    algo.train(mem)
    torch.manual_seed(8)
    R.train(ref, ref_mem, 0)
    p_eng, p_ref = agent.packed_params().cpu(), R.flat_params(ref)
    close = (p_eng - p_ref).abs() <= 1e-5 * p_ref.abs() + 1e-7
    assert float(close.float().mean()) >= 0.99
    assert float((p_eng - p_ref).abs().max()) <= 2.5e-4


def test_philox_mode_runs_and_is_reproducible(gpu):
    outs = []
    for _ in range(2):
        algo, agent, *_ = _setup(gpu, n=64, t=32, b=512, epochs=2, rng="philox", seed=3)
        before = agent.flat_params.clone()
        algo.iterate(verbose=False)
        assert all(map(lambda x: x == x, algo.last_losses))
        assert not torch.equal(before, agent.flat_params)
        outs.append(agent.packed_params().cpu().clone())
    assert torch.equal(outs[0], outs[1]), "philox mode must be bit-reproducible"


@pytest.mark.parametrize("prec,hidden,n,b", [("f32", (64, 64), 64, 256),
                                             ("bf16", (256, 256), 128, 512)])
def test_graphs_match_eager(gpu, prec, hidden, n, b):
    """rollout_graph / train_graph (each captured once, replayed with the device Philox counter,
    the pre-drawn minibatch rows and the device Adam schedule) produce the same buffers and
    parameters, bit for bit, as the eager launch sequence over 3 iterations (iteration 0 eager
    warm-up, 1 capture + replay, 2 replay).  bf16 at 2x256 runs the fused kernels."""
    res = []
    for graph in (False, True):
        algo, agent, *_ = _setup(gpu, n=n, t=16, b=b, epochs=2, hidden=hidden, rng="philox",
                                 seed=4, rollout_graph=graph, train_graph=graph, precision=prec)
        snaps = []
        for _ in range(3):
            algo.iterate(verbose=False)
            torch.cuda.synchronize()
            snaps.append((algo.buffer.actions.cpu().clone(), algo.buffer.logp.cpu().clone(),
                          algo.buffer.states.cpu().clone(), agent.packed_params().cpu().clone(),
                          agent.flat_m.cpu().clone(), agent.flat_v.cpu().clone(),
                          torch.tensor(algo.last_losses)))
        assert (algo._graph is not None) == graph
        assert (getattr(algo, "_tg_graph", None) is not None) == graph
        assert agent.optimizers["actor"].step_count == 3 * 2 * (n * 16 // b)
        res.append(snaps)
    names = ("actions", "logp", "states", "params", "adam m", "adam v", "losses")
    for it, (e, g) in enumerate(zip(*res)):
        for name, x, y in zip(names, e, g):
            assert torch.equal(x, y), f"iteration {it}: {name} differs between graph and eager"
    # fresh noise every iteration (the counter advanced)
    assert not torch.equal(res[1][1][0], res[1][2][0])


def test_bf16_iteration_tracks_f32(gpu):
    """precision="bf16" (BASELINE configs[1]): one PPO iteration from the same init and the same
    Philox streams moves the parameters in nearly the same direction as the f32 engine: the two
    updates (post - init) agree to 10 % in relative L2, rollout values to 2e-2 relative."""
    out = {}
    for prec in ("f32", "bf16"):
        algo, agent, *_ = _setup(gpu, n=256, t=32, b=2048, epochs=2, hidden=(256, 256),
                                 rng="philox", seed=6, precision=prec)
        p0 = agent.packed_params().clone()
        algo.iterate(verbose=False)
        assert all(map(lambda x: x == x, algo.last_losses))
        out[prec] = (agent.packed_params() - p0, algo.buffer.values.clone())
    du_f, v_f = out["f32"]
    du_b, v_b = out["bf16"]
    rel = float((du_b - du_f).norm() / du_f.norm())
    assert rel < 0.1, rel
    vrel = float((v_b - v_f).abs().max() / v_f.abs().max())
    assert vrel < 2e-2, vrel


def test_headline_shape_iteration_smoke(gpu):
    """The bench workload's shapes (N=4096, T=128, 2x256, B=65536) for one epoch."""
    algo, agent, *_ = _setup(gpu, n=4096, t=128, b=65536, epochs=1, hidden=(256, 256),
                             rng="philox", p_term=0.0)
    algo.iterate(verbose=False)
    assert all(abs(x) < 1e6 for x in algo.last_losses)
    adv = algo.buffer.advantage
    assert bool(torch.isfinite(adv).all())


def test_checkpoint_roundtrip(gpu, tmp_path):
    algo, agent, *_ = _setup(gpu, experiment_path=str(tmp_path))
    algo.iterate(verbose=False)
    agent.run.dynamic_config.current_episode = 3
    agent.save()
    saved = agent.packed_params().clone()
    m_saved = agent.packed(agent.flat_m).clone()
    agent.flat_params.add_(1.0)
    agent.flat_m.zero_()
    agent.load()
    assert torch.equal(agent.packed_params(), saved)
    assert torch.equal(agent.packed(agent.flat_m), m_saved)
    sd = torch.load(tmp_path / "networks" / "3" / "networks.pth", weights_only=True)
    assert "actor.actor.first_layers.0.weight" in sd and "critic.network.last_layer.bias" in sd


@pytest.mark.parametrize("prec,hidden", [("f32", (64, 64)), ("bf16", (256, 256))])
def test_host_physics_pool_matches_device_env(gpu, prec, hidden):
    """HostPhysicsVecEnvHelper (P=2 worker processes, page-locked shared memory, hipMemcpyAsync
    on a side stream) drives two PPO iterations to the same rollout buffers, losses and
    parameters, bit for bit, as the device-resident synthetic env on the same streams."""
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (HostPhysicsVecEnvHelper,
                                                                SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    n, t, b = 96, 16, 512
    streams = make_synthetic_streams(n, t, 17, seed=9, p_terminate=0.05)
    res = []
    for cls in (SyntheticVecEnvHelper, HostPhysicsVecEnvHelper):
        run = make_run(num_envs=n, horizon=t, hidden=hidden, batch_size=b, epochs=2, rng="philox",
                       seed=2, precision=prec)
        torch.manual_seed(2)
        agent = PPOEngineAgent(run, device=gpu)
        kw = {"workers": 2} if cls is HostPhysicsVecEnvHelper else {}
        helper = cls(streams, run, device=gpu, **kw)
        algo = PPOEngine(helper, agent, log=lambda m: None)
        snaps = []
        for _ in range(2):
            algo.iterate(verbose=False)
            torch.cuda.synchronize()
            buf = algo.buffer
            snaps.append([x.cpu().clone() for x in (buf.states, buf.actions, buf.reward,
                                                   buf.terminated, buf.values, buf.advantage,
                                                   agent.packed_params())])
        if cls is HostPhysicsVecEnvHelper:
            helper.close()
        res.append(snaps)
    names = ("states", "actions", "reward", "terminated", "values", "advantage", "params")
    for it, (d, h) in enumerate(zip(*res)):
        for name, x, y in zip(names, d, h):
            assert torch.equal(x, y), f"iteration {it}: {name} differs (host pool vs device env)"
