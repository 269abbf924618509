"""GPU parity of each hot-path kernel against the CPU oracle (oracle/ppo_ref.py).

Bars (written next to each check): bit-exact for GAE (f64 carry), the minibatch row maps, the
synthetic env, the sampling arithmetic given (eps, mean, std) and Adam given identical grads;
tolerances for the MLP (f32 GEMM summation order differs from CPU MKL) and for transcendental
functions (device vs SLEEF tanh/exp/log, <= a few ulp).
"""
import numpy as np
import pytest
import torch

from oracle import ppo_ref as R

pytestmark = pytest.mark.gpu


def _E():
    from mujoco_reinforcement_learning_amd import engine as E
    return E


# ---------------------------------------------------------------------------------- GAE (A7/A8)
@pytest.mark.parametrize("kernel", ["pipe", "chain"])
@pytest.mark.parametrize("n,t,p_term,reward_f64", [(8, 16, 0.1, True), (257, 33, 0.05, True),
                                                   (4096, 128, 0.0, True), (1000, 64, 0.2, False),
                                                   (3, 1, 0.5, True), (16384, 128, 0.01, True),
                                                   (100, 200, 0.02, True)])
def test_gae_bit_exact(gpu, monkeypatch, n, t, p_term, reward_f64, kernel):
    """kernel: the pipelined scan (gae_pipe_kernel, the default) or the producer / consumer one
    (gae_chain_kernel, opt-in) -- both bit-exact against the oracle's f64 recurrence."""
    monkeypatch.setenv("PPO_GAE_KERNEL", kernel)
    E = _E()
    g = torch.Generator().manual_seed(n * 7 + t)
    v = torch.randn(n, t, 1, generator=g)
    vn = torch.randn(n, t, 1, generator=g)
    rdt = torch.float64 if reward_f64 else torch.float32
    r = torch.randn(n, t, 1, generator=g, dtype=rdt)
    term = torch.rand(n, t, 1, generator=g) < p_term
    done = term.clone()
    done[:, -1] = True
    adv_ref, vt_ref = R.generalized_advantage_estimate(0.99, 0.98, v, vn, r, done, term)
    tm = lambda x: x[..., 0].t().contiguous().to(gpu)  # (N,T,1) -> time-major (T,N)
    adv = torch.empty(t, n, device=gpu)
    vt = torch.empty(t, n, device=gpu)
    E.gae(tm(v), tm(vn), tm(r), tm(term), 0.99, 0.98, adv, vt, force_last_done=True)
    assert torch.equal(adv.t().cpu(), adv_ref[..., 0]), "GAE advantage not bit-exact"
    assert torch.equal(vt.t().cpu(), vt_ref[..., 0]), "GAE value target not bit-exact"


@pytest.mark.parametrize("kernel", ["pipe", "chain"])
def test_gae_explicit_done_and_nan_propagation(gpu, monkeypatch, kernel):
    monkeypatch.setenv("PPO_GAE_KERNEL", kernel)
    E = _E()
    n, t = 64, 20
    g = torch.Generator().manual_seed(1)
    v = torch.randn(n, t, 1, generator=g)
    vn = torch.randn(n, t, 1, generator=g)
    vn[3, 5, 0] = float("nan")
    r = torch.randn(n, t, 1, generator=g, dtype=torch.float64)
    term = torch.rand(n, t, 1, generator=g) < 0.1
    done = term | (torch.rand(n, t, 1, generator=g) < 0.1)  # truncation-style dones
    adv_ref, vt_ref = R.generalized_advantage_estimate(0.9, 0.7, v, vn, r, done, term)
    tm = lambda x: x[..., 0].t().contiguous().to(gpu)
    adv = torch.empty(t, n, device=gpu)
    vt = torch.empty(t, n, device=gpu)
    E.gae(tm(v), tm(vn), tm(r), tm(term), 0.9, 0.7, adv, vt, done=tm(done), force_last_done=False)
    a = adv.t().cpu()
    assert torch.equal(torch.isnan(a), torch.isnan(adv_ref[..., 0]))
    ok = ~torch.isnan(a)
    assert torch.equal(a[ok], adv_ref[..., 0][ok])


# ------------------------------------------------------------------------- normalisation (A6/A9)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_normalize_rows(gpu, dtype):
    E = _E()
    n, t = 300, 128
    g = torch.Generator().manual_seed(2)
    x = (torch.randn(n, t, 1, generator=g) * 3 + 1).to(dtype)
    ref = x - x.mean(dim=1).unsqueeze(1)
    ref = (ref / ref.std(dim=1).unsqueeze(1)) * 1.0
    xt = x[..., 0].t().contiguous().to(gpu)
    E.normalize_rows(xt, 1.0)
    tol = dict(rtol=2e-6, atol=2e-6) if dtype == torch.float32 else dict(rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(xt.t().cpu(), ref[..., 0], **tol)


# ---------------------------------------------------------------------- observations (A1) + env
@pytest.mark.parametrize("o,w", [(17, 1), (17, 3), (27, 2), (376, 1), (376, 2)])
def test_obs_window_and_normalize(gpu, o, w):
    E = _E()
    n = 50
    g = torch.Generator().manual_seed(o + w)
    first = torch.randn(n, o, generator=g)
    win_ref = first.double()[..., None].repeat(1, 1, w)
    win = torch.zeros(n, o, w, dtype=torch.float64, device=gpu)
    E.obs_window_push(win, first.to(gpu), all_reset=True)
    for k in range(3):
        nxt = torch.randn(n, o, generator=g, dtype=torch.float64)
        reset = torch.rand(n, generator=g) < 0.3
        shifted = torch.cat([win_ref[:, :, 1:], nxt[..., None]], dim=2)
        win_ref = torch.where(reset[:, None, None], nxt[..., None].repeat(1, 1, w), shifted)
        E.obs_window_push(win, nxt.to(gpu), reset=reset.to(gpu))
    assert torch.equal(win.cpu(), win_ref)
    st = torch.empty(n, w, o, device=gpu)
    E.obs_normalize(win, st)
    ref = R.get_state(win_ref, True)
    # f64 statistics, rounded once to f32: equal except (rare) f64 summation-order ties
    diff = (st.cpu() - ref).abs()
    ulp = torch.finfo(torch.float32).eps * ref.abs().clamp_min(1e-30)
    assert bool((diff <= ulp).all()), float((diff / ulp).max())
    E.obs_normalize(win, st, normalize=False)
    assert torch.equal(st.cpu(), win_ref.float().permute(0, 2, 1))


def test_synthetic_env_step_bit_exact(gpu):
    E = _E()
    n, o, a, t = 40, 17, 6, 4
    g = torch.Generator().manual_seed(4)
    base_obs = torch.randn(t + 1, n, o, generator=g)
    base_r = torch.rand(t, n, generator=g) * 2 - 1
    base_term = torch.rand(t, n, generator=g) < 0.3
    env = R.RefSyntheticEnv(base_obs, base_r, base_term, 1, a)
    env.reset()
    act = torch.randn(n, a, generator=g)
    env.step(act)
    obs = torch.empty(n, o, dtype=torch.float64, device=gpu)
    rew = torch.empty(n, dtype=torch.float64, device=gpu)
    term = torch.empty(n, dtype=torch.bool, device=gpu)
    E.synthetic_env_step(base_obs[1].to(gpu), base_r[0].to(gpu), base_term[0].to(gpu), act.to(gpu),
                         obs, rew, term)
    assert torch.equal(obs.cpu(), env.window[..., -1])
    assert torch.equal(rew.cpu(), env.reward)
    assert torch.equal(term.cpu(), env.terminated)


# --------------------------------------------------------------------------- RNG + rows (A10)
def test_philox_normals_deterministic_and_standard(gpu):
    E = _E()
    x = torch.empty(1 << 20, device=gpu)
    E.philox_normal(7, 0, x)
    y = torch.empty(1 << 20, device=gpu)
    E.philox_normal(7, 0, y)
    assert torch.equal(x, y)
    z = torch.empty(1000, device=gpu)
    E.philox_normal(7, 5000, z)
    assert torch.equal(z, x[5000:6000])
    assert abs(float(x.mean())) < 5e-3 and abs(float(x.std()) - 1) < 5e-3


def test_perm_to_rows_bit_exact_and_shard(gpu):
    E = _E()
    n, t, b = 64, 32, 500
    torch.manual_seed(0)
    perm = torch.randperm(n * t)
    rows = torch.empty(b, dtype=torch.int32, device=gpu)
    E.perm_to_rows(perm.to(gpu), 700, b, n, t, rows)
    f = perm[700:700 + b]
    assert torch.equal(rows.cpu().long(), (f % t) * n + f // t)
    # exact-DP shard [16, 40): kept in order, rank-local time-major rows
    cnt = torch.zeros(1, dtype=torch.int32, device=gpu)
    E.perm_to_rows(perm.to(gpu), 700, b, n, t, rows, shard=(16, 40), count=cnt)
    env = f // t
    keep = (env >= 16) & (env < 40)
    exp = (f[keep] % t) * 24 + (env[keep] - 16)
    assert int(cnt) == int(keep.sum())
    assert torch.equal(rows[:int(cnt)].cpu().long(), exp)


def test_feistel_rows_is_a_permutation(gpu):
    E = _E()
    n, t = 4096, 128
    rows = torch.empty(n * t, dtype=torch.int32, device=gpu)
    E.feistel_rows(123, 4, 0, n * t, n, t, rows)
    assert torch.equal(torch.sort(rows.long()).values.cpu(), torch.arange(n * t))
    rows2 = torch.empty_like(rows)
    E.feistel_rows(123, 5, 0, n * t, n, t, rows2)
    assert not torch.equal(rows, rows2)


# --------------------------------------------------------------------------------- Adam (A15)
def test_adam_matches_torch_adam(gpu):
    """Same grads in -> torch.optim.Adam (CPU single-tensor path) out, over several steps."""
    E = _E()
    n = 4099
    g = torch.Generator().manual_seed(5)
    p = torch.randn(n, generator=g)
    m = torch.zeros(n)
    v = torch.zeros(n)
    pd, md, vd = p.to(gpu), m.to(gpu), v.to(gpu)
    lr = 1e-4
    worst = 0
    for step in range(1, 6):
        grad = torch.randn(n, generator=g) * (10.0 ** (-step))
        p, m, v = R.adam_reference_step(p, grad, m, v, step, lr)
        bc1 = 1 - 0.9 ** step
        bc2 = (1 - 0.999 ** step) ** 0.5
        E.adam(pd, grad.to(gpu), md, vd, 1000, -lr / bc1, -lr / bc1, 1 - 0.9, 0.999, 1 - 0.999,
               bc2, 1e-8)
        worst = max(worst, int((pd.cpu() != p).sum()))
        assert torch.equal(md.cpu(), m), "exp_avg (lerp) not bit-exact"
        assert torch.equal(vd.cpu(), v), "exp_avg_sq not bit-exact"
    # param: bit-exact on the vectorised body; torch's scalar tail may round 1 ulp apart
    torch.testing.assert_close(pd.cpu(), p, rtol=0, atol=2 * torch.finfo(torch.float32).eps)
    assert worst <= n // 100


# -------------------------------------------------------------------- policy step (A2-A4)
def _agents(gpu, seed, **kw):
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    run = make_run(**kw)
    torch.manual_seed(seed)
    eng = PPOEngineAgent(run, device=gpu)
    cfg = R.RefConfig(num_envs=run.environment_config.num_envs,
                      horizon=run.environment_config.maximum_timesteps,
                      obs_dim=run.network_config.input_shape, act_dim=run.network_config.output_shape,
                      window=run.environment_config.window_length,
                      actor_hidden=tuple(run.network_config.linear_hidden_shapes),
                      critic_hidden=tuple(run.engine_config.critic_hidden_shapes or
                                          run.network_config.linear_hidden_shapes),
                      activation=kw.get("activation", "relu"),
                      batch_size=int(run.training_config.batch_size),
                      epochs=run.training_config.epochs_per_iteration,
                      normalize_advantage=run.ppo_config.normalize_advantage,
                      normalize_rewards=run.normalize_rewards)
    torch.manual_seed(seed)
    ref = R.RefAgent(cfg)
    return run, eng, ref, cfg


@pytest.mark.parametrize("hidden,act,n,window", [((64, 64), "relu", 64, 1),
                                                 ((256, 256), "relu", 4096, 1),
                                                 ((64, 64), "tanh", 100, 2),
                                                 ((512, 512, 512), "elu", 300, 1)])
def test_policy_step_matches_oracle(gpu, hidden, act, n, window):
    run, eng, ref, cfg = _agents(gpu, 3, num_envs=n, hidden=hidden, activation=act, window=window,
                                 batch_size=n)
    assert torch.equal(eng.packed_params().cpu(), R.flat_params(ref)), "init differs from oracle"
    g = torch.Generator().manual_seed(9)
    state = torch.randn(n, window, 17, generator=g)
    eps = torch.randn(n, 6, generator=g)
    sd = state.reshape(n, -1).contiguous().to(gpu)
    action = torch.empty(n, 6, device=gpu)
    mean = torch.empty(n, 6, device=gpu)
    logp = torch.empty(n, device=gpu)
    value = torch.empty(n, device=gpu)
    eng.engine.policy_step(sd, eps=eps.to(gpu), action=action, logp=logp, value=value, mean=mean)
    with torch.no_grad():
        m_ref, s_ref = ref.networks["actor"](state)
        v_ref = ref.networks["critic"](state)[:, 0]
    torch.testing.assert_close(mean.cpu(), m_ref, rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(value.cpu(), v_ref, rtol=1e-5, atol=2e-6)
    # sampling arithmetic: fl(fl(eps*std) + mean) on the engine's own mean/std -> bit-exact
    std = eng.networks["actor"].actor_logstd.detach().exp().cpu()
    assert torch.equal(action.cpu(), eps * std + mean.cpu())
    lp_ref = torch.distributions.Normal(mean.cpu(), s_ref).log_prob(action.cpu()).sum(dim=1)
    torch.testing.assert_close(logp.cpu(), lp_ref, rtol=1e-6, atol=1e-5)


# ---------------------------------------------------------------- minibatch gradients (A11-A13)
@pytest.mark.parametrize("hidden,act,rows_total,b", [((64, 64), "relu", 512, 128),
                                                     ((256, 256), "relu", 8192, 4096),
                                                     ((64, 32), "tanh", 300, 100)])
def test_minibatch_grad_matches_autograd(gpu, hidden, act, rows_total, b):
    run, eng, ref, cfg = _agents(gpu, 4, num_envs=rows_total, hidden=hidden, activation=act,
                                 batch_size=b)
    g = torch.Generator().manual_seed(10)
    states = torch.randn(rows_total, 17, generator=g)
    actions = torch.randn(rows_total, 6, generator=g) * 0.5
    old_logp = torch.randn(rows_total, generator=g) - 6.0
    adv = torch.randn(rows_total, generator=g)
    vt = torch.randn(rows_total, generator=g)
    # make some ratios land outside the clip range and on both sides of the Huber knee
    with torch.no_grad():
        m_ref, s_ref = ref.networks["actor"](states)
        lp = torch.distributions.Normal(m_ref, s_ref).log_prob(actions).sum(1)
    old_logp = lp + torch.randn(rows_total, generator=g) * 0.2
    vt = vt * 2
    rows = torch.randperm(rows_total, generator=g)[:b].to(torch.int32)
    grad = torch.empty(eng.engine.n_params, device=gpu)
    loss = torch.empty(2, device=gpu)
    eng.engine.minibatch_grad(states.to(gpu), actions.to(gpu), old_logp.to(gpu), adv.to(gpu),
                              vt.to(gpu), rows.to(gpu), b, grad, loss, 0.9, 1.1, 1e-4, 1.0 / b,
                              1.0 / (b * 6))
    # oracle: the ppo.py:110-135 losses on the same rows, torch autograd
    idx = rows.long()
    x = states[idx][:, None, :]
    _, dist = ref.act(x, return_dist=True)
    new_lp = dist.log_prob(actions[idx]).sum(dim=1)
    v = ref.get_state_value(x)
    lc = torch.nn.functional.huber_loss(v, vt[idx][:, None], reduction="mean")
    ent = dist.entropy().mean()
    ratio = (new_lp - old_logp[idx]).exp()[:, None]
    a_ = adv[idx][:, None]
    la = -torch.min(ratio * a_, torch.clamp(ratio, 0.9, 1.1) * a_).mean() - ent * 1e-4
    ref.networks.zero_grad()
    (la + lc).backward()
    gref = torch.cat([p.grad.flatten() for p in ref.networks.parameters()])
    gd = eng.packed(grad).cpu()
    off = 0
    for name, p in ref.networks.named_parameters():
        k = p.numel()
        a, r_ = gd[off:off + k], gref[off:off + k]
        scale = float(r_.abs().max()) + 1e-12
        err = float((a - r_).abs().max())
        assert err <= 2e-5 * scale + 1e-9, (name, err, scale)
        off += k
    torch.testing.assert_close(loss.cpu()[1], lc.detach(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(loss.cpu()[0], la.detach(), rtol=1e-4, atol=1e-6)


def test_per_kernel_timing_records(gpu):
    """ppo_ctx_timing_kernel: one record per kernel instantiation, named as rocprofv3 spells it,
    covering ctx entry points (GEMMs, heads) and ctx-free ones (GAE, Adam) while enabled."""
    E = _E()
    run, eng, ref, cfg = _agents(gpu, 4, num_envs=256, hidden=(64, 64), activation="relu",
                                 batch_size=128)
    g = torch.Generator().manual_seed(3)
    n = 256
    states = torch.randn(n, 17, generator=g).to(gpu)
    actions = torch.randn(n, 6, generator=g).to(gpu)
    vec = [torch.randn(n, generator=g).to(gpu) for _ in range(3)]
    rows = torch.randperm(n, generator=g)[:128].to(torch.int32).to(gpu)
    grad = torch.empty(eng.engine.n_params, device=gpu)
    loss = torch.empty(2, device=gpu)
    eng.engine.timing(True, capacity=1024)
    eng.engine.minibatch_grad(states, actions, vec[0], vec[1], vec[2], rows, 128, grad, loss,
                              0.9, 1.1, 1e-4, 1.0 / 128, 1.0 / (128 * 6))
    v = torch.randn(16, 32, device=gpu)
    r = torch.randn(16, 32, device=gpu, dtype=torch.float64)
    term = torch.zeros(16, 32, device=gpu, dtype=torch.bool)
    adv, vt = torch.empty_like(v), torch.empty_like(v)
    E.gae(v, v, r, term, 0.99, 0.98, adv, vt)
    kernels = eng.engine.timing_kernels()
    eng.engine.timing(False)
    classes = {rec["class"] for rec in kernels.values()}
    assert {"gemm_fwd", "gemm_wgrad", "gemm_dgrad", "update_head", "reduce_slabs",
            "gather_states", "gae"} <= classes, classes
    gemms = [k for k, rec in kernels.items() if rec["class"].startswith("gemm")]
    assert all(k.startswith("gemm_f32_kernel<") and k.count(",") == 10 for k in gemms), gemms
    for k, rec in kernels.items():
        assert rec["launches"] >= 1 and rec["ms"] > 0.0, (k, rec)
    gae = [rec for rec in kernels.values() if rec["class"] == "gae"]
    assert len(gae) == 1 and gae[0]["bytes"] == 16 * 32 * 25
    # disabled timing records nothing further
    E.gae(v, v, r, term, 0.99, 0.98, adv, vt)
    assert eng.engine.timing_kernels() == kernels


# ------------------------------------------------------------- bf16 GEMM precision mode
@pytest.mark.parametrize("hidden,act,rows_total,b,obs,na", [
    ((64, 64), "relu", 512, 128, 17, 6),
    ((256, 256), "relu", 8192, 4096, 17, 6),        # fused kernel (fused_update.hip) from here on
    ((256, 256), "tanh", 3000, 1000, 17, 6),        # ragged last chunk (1000 = 15*64 + 40)
    ((256, 256), "elu", 2000, 300, 27, 8),          # Ant-v4 shapes (O=27, A=8)
    ((256, 256), "relu", 70000, 65536, 17, 6),      # bench minibatch: 128 workgroups x 8 chunks
    ((64, 32), "tanh", 300, 100, 17, 6)])
def test_minibatch_grad_bf16_matches_emulation(gpu, hidden, act, rows_total, b, obs, na):
    """precision="bf16": every hidden fc GEMM (forward, dgrad, wgrad) takes bf16-rounded operands
    with f32 accumulation.  Checked against torch autograd on the oracle nets with the same
    operand rounding (oracle.use_bf16_gemms); the residual is f32 summation order plus
    rare bf16 rounding-boundary flips of intermediates, so the bound is relative, 2e-3 of each
    tensor's largest gradient.  Against plain f32 autograd each tensor is within 10 % relative
    L2 (bf16 operand noise)."""
    run, eng, ref, cfg = _agents(gpu, 4, num_envs=rows_total, hidden=hidden, activation=act,
                                 batch_size=b, precision="bf16", obs_dim=obs, act_dim=na)
    assert eng.engine.precision == "bf16"
    g = torch.Generator().manual_seed(10)
    states = torch.randn(rows_total, obs, generator=g)
    actions = torch.randn(rows_total, na, generator=g) * 0.5
    adv = torch.randn(rows_total, generator=g)
    vt = torch.randn(rows_total, generator=g) * 2
    with torch.no_grad():
        m_ref, s_ref = ref.networks["actor"](states)
        lp = torch.distributions.Normal(m_ref, s_ref).log_prob(actions).sum(1)
    old_logp = lp + torch.randn(rows_total, generator=g) * 0.2
    rows = torch.randperm(rows_total, generator=g)[:b].to(torch.int32)
    grad = torch.empty(eng.engine.n_params, device=gpu)
    loss = torch.empty(2, device=gpu)
    eng.engine.timing(True)
    eng.engine.minibatch_grad(states.to(gpu), actions.to(gpu), old_logp.to(gpu), adv.to(gpu),
                              vt.to(gpu), rows.to(gpu), b, grad, loss, 0.9, 1.1, 1e-4, 1.0 / b,
                              1.0 / (b * na))
    kernels = eng.engine.timing_kernels()
    eng.engine.timing(False)
    fused = hidden == (256, 256)
    assert any(k.startswith("fused_update_kernel<256") for k in kernels) == fused, kernels
    # the fused kernel launches no layered GEMMs (ReLU nets off the fused shapes take the wide
    # bf16-resident path, wide_engine.hip; the others the layered gemm_ kernels)
    assert (not any(k.startswith(("gemm_", "wide_gemm_")) for k in kernels)) == fused, kernels
    gd = eng.packed(grad).cpu()

    def ref_grad(bf16: bool):
        import copy
        r = copy.deepcopy(ref)
        if bf16:
            R.use_bf16_gemms(r)
        idx = rows.long()
        x = states[idx][:, None, :]
        _, dist = r.act(x, return_dist=True)
        new_lp = dist.log_prob(actions[idx]).sum(dim=1)
        v = r.get_state_value(x)
        lc = torch.nn.functional.huber_loss(v, vt[idx][:, None], reduction="mean")
        ratio = (new_lp - old_logp[idx]).exp()[:, None]
        a_ = adv[idx][:, None]
        la = -torch.min(ratio * a_, torch.clamp(ratio, 0.9, 1.1) * a_).mean() \
            - dist.entropy().mean() * 1e-4
        r.networks.zero_grad()
        (la + lc).backward()
        losses.append((float(la), float(lc)))
        return [(n, p.grad.flatten().clone()) for n, p in r.networks.named_parameters()]

    losses = []
    off = 0
    for name, r_ in ref_grad(True):
        k = r_.numel()
        a = gd[off:off + k]
        scale = float(r_.abs().max()) + 1e-12
        err = float((a - r_).abs().max())
        assert err <= 2e-3 * scale + 1e-9, (name, err, scale)
        off += k
    off = 0
    for name, r_ in ref_grad(False):  # plain f32: relative L2 per tensor within bf16 noise
        k = r_.numel()
        a = gd[off:off + k]
        rel = float((a - r_).norm() / (r_.norm() + 1e-12))
        assert rel <= 0.1, (name, rel)
        off += k
    # loss scalars (actor: surrogate + entropy, critic: Huber) against the bf16 emulation
    la_ref, lc_ref = losses[0]
    got = loss.cpu()
    assert abs(float(got[0]) - la_ref) <= 1e-3 * (abs(la_ref) + 1e-2), (float(got[0]), la_ref)
    assert abs(float(got[1]) - lc_ref) <= 1e-3 * (abs(lc_ref) + 1e-2), (float(got[1]), lc_ref)


# ------------------------------------------------------------- fused observe + act (A1-A4)
@pytest.mark.parametrize("act,n,window,obs,na,reset_p", [("relu", 4096, 1, 17, 6, 0.0),
                                                          ("tanh", 1000, 1, 17, 6, 0.1),
                                                          ("elu", 300, 1, 27, 8, 0.5),
                                                          ("relu", 77, 1, 11, 3, 0.3)])
def test_observe_act_fused_matches_layered(gpu, act, n, window, obs, na, reset_p):
    """precision="bf16", 2x256: ppo_observe_act (one fused launch: window push, f64
    standardisation, both MLPs on bf16 MFMA, heads, sampling) against the A1 kernels + the
    layered bf16 policy_step on the same context.  Window and state are bit-exact (same f64
    arithmetic); actions / log-probs / values agree to f32 summation order of identical
    bf16-operand products (rtol 2e-4 relative to each output's scale)."""
    E = _E()
    run, eng, ref, cfg = _agents(gpu, 7, num_envs=n, hidden=(256, 256), activation=act,
                                 batch_size=n, precision="bf16", obs_dim=obs, act_dim=na)
    e = eng.engine
    g = torch.Generator().manual_seed(n + obs)
    win0 = torch.randn(n, obs, window, generator=g, dtype=torch.float64)
    new_obs = torch.randn(n, obs, generator=g, dtype=torch.float64)
    reset = (torch.rand(n, generator=g) < reset_p).to(torch.uint8)
    eps = torch.randn(n, na, generator=g)
    outs = {}
    for mode in ("fused", "layered"):
        win = win0.clone().to(gpu)
        st = torch.empty(n, window * obs, device=gpu)
        act_, lp, val, mu = (torch.empty(n, na, device=gpu), torch.empty(n, device=gpu),
                             torch.empty(n, device=gpu), torch.empty(n, na, device=gpu))
        if mode == "fused":
            e.pack_weights()
            e.observe_act(win, st, obs=new_obs.to(gpu), reset=reset.to(gpu), eps=eps.to(gpu),
                          action=act_, logp=lp, value=val, mean=mu)
        else:
            E.obs_window_push(win, new_obs.to(gpu), reset=reset.to(gpu))
            E.obs_normalize(win, st)
            e.policy_step(st, eps=eps.to(gpu), action=act_, logp=lp, value=val, mean=mu)
        torch.cuda.synchronize()
        outs[mode] = [x.cpu() for x in (win, st, act_, lp, val, mu)]
    f, l = outs["fused"], outs["layered"]
    assert torch.equal(f[0], l[0]), "window push differs"
    assert torch.equal(f[1], l[1]), "standardised state differs"
    for name, a, b in zip(("action", "logp", "value", "mean"), f[2:], l[2:]):
        scale = float(b.abs().max()) + 1e-6
        err = float((a - b).abs().max())
        assert err <= 2e-4 * scale, (name, err, scale)
    # value-only call (t = T; only the critic's workgroups run, and they write window + state)
    # and action-only call
    win = win0.clone().to(gpu)
    st = torch.full((n, window * obs), float("nan"), device=gpu)
    val = torch.full((n,), float("nan"), device=gpu)
    e.observe_act(win, st, obs=new_obs.to(gpu), reset=reset.to(gpu), value=val)
    assert torch.allclose(val.cpu(), l[4], rtol=0, atol=2e-4 * (float(l[4].abs().max()) + 1e-6))
    assert torch.equal(win.cpu(), l[0]), "value-only call: window push differs"
    assert torch.equal(st.cpu(), l[1]), "value-only call: state differs"
    win = win0.clone().to(gpu)
    act_ = torch.full((n, na), float("nan"), device=gpu)
    e.observe_act(win, st, obs=new_obs.to(gpu), reset=reset.to(gpu), eps=eps.to(gpu), action=act_)
    assert torch.isfinite(act_).all()


@pytest.mark.parametrize("hidden,n,window,obs,na,reset_p", [
    ((512, 512, 512), 1024, 1, 376, 17, 0.0),   # Humanoid-v4 shard (its six slices)
    ((512, 512, 512), 77, 1, 376, 17, 0.3),     # ragged: padding operand rows
    ((64, 64), 300, 3, 27, 8, 0.3)])            # window of 3 (push shifts the kept slots)
def test_observe_act_wide_matches_layered(gpu, hidden, n, window, obs, na, reset_p):
    """precision="bf16", ReLU nets off the fused shapes (the wide path): ppo_observe_act (one
    wide_observe_kernel launch: window push, f64 standardisation, bf16 operand rows; then the
    wide GEMMs) against ppo_obs_window_push + ppo_obs_normalize + policy_step (which stages the
    rows itself) on the same context: window, state and every output bit for bit."""
    E = _E()
    run, eng, ref, cfg = _agents(gpu, 5, num_envs=n, hidden=hidden, batch_size=n,
                                 precision="bf16", obs_dim=obs, act_dim=na, window=window)
    e = eng.engine
    g = torch.Generator().manual_seed(n + obs + window)
    win0 = torch.randn(n, obs, window, generator=g, dtype=torch.float64) * 3 + 1
    new_obs = torch.randn(n, obs, generator=g, dtype=torch.float64) * 3 + 1
    reset = (torch.rand(n, generator=g) < reset_p).to(torch.uint8)
    eps = torch.randn(n, na, generator=g)
    e.pack_weights()
    outs = {}
    for mode in ("observe_act", "layered"):
        win = win0.clone().to(gpu)
        st = torch.full((n, window * obs), float("nan"), device=gpu)
        act_, lp, val, mu = (torch.empty(n, na, device=gpu), torch.empty(n, device=gpu),
                             torch.empty(n, device=gpu), torch.empty(n, na, device=gpu))
        e.timing(True)
        if mode == "observe_act":
            e.observe_act(win, st, obs=new_obs.to(gpu), reset=reset.to(gpu), eps=eps.to(gpu),
                          action=act_, logp=lp, value=val, mean=mu)
        else:
            E.obs_window_push(win, new_obs.to(gpu), reset=reset.to(gpu))
            E.obs_normalize(win, st)
            e.policy_step(st, eps=eps.to(gpu), action=act_, logp=lp, value=val, mean=mu)
        torch.cuda.synchronize()
        kernels = e.timing_kernels()
        e.timing(False)
        assert ("wide_observe_kernel" in kernels) == (mode == "observe_act"), kernels
        # the fused rollout kernel when the widths allow it, else the layered GEMMs
        assert ("wide_policy_fused_kernel" in kernels or
                any(k.startswith("wide_gemm_kernel") for k in kernels)), kernels
        outs[mode] = [x.cpu() for x in (win, st, act_, lp, val, mu)]
    for name, a, b in zip(("window", "state", "action", "logp", "value", "mean"),
                          outs["observe_act"], outs["layered"]):
        assert torch.equal(a, b), f"{name} differs between observe_act and the layered calls"


@pytest.mark.parametrize("n", [1024, 77])
def test_policy_step_wide_fused_matches_layered(gpu, monkeypatch, n):
    """Humanoid shapes (3x512, O=376, A=17), bf16: the fused rollout kernel
    (wide_policy_fused_kernel: hidden layers, heads, sampling in one launch) against the layered
    wide rollout (FWD GEMMs + head GEMM + wide_policy_head_kernel; PPO_WIDE_FUSED_ROLLOUT=0) on
    the same parameters and noise.  Both sum every product in the same k order on the same bf16
    operands; the bar allows for the MFMA computing W.act^T instead of act.W^T: mean / value
    within 1e-6 of their scale, actions fl(fl(eps*std)+mean) of each one's own mean, log-prob
    within 1e-5."""
    outs = {}
    for mode in ("layered", "fused"):
        monkeypatch.setenv("PPO_WIDE_FUSED_ROLLOUT", "1" if mode == "fused" else "0")
        run, eng, ref, cfg = _agents(gpu, 3, num_envs=n, hidden=(512, 512, 512), batch_size=n,
                                     precision="bf16", obs_dim=376, act_dim=17)
        e = eng.engine
        g = torch.Generator().manual_seed(5)
        state = torch.randn(n, 376, generator=g).to(gpu)
        eps = torch.randn(n, 17, generator=g).to(gpu)
        act_, lp, val, mu = (torch.empty(n, 17, device=gpu), torch.empty(n, device=gpu),
                             torch.empty(n, device=gpu), torch.empty(n, 17, device=gpu))
        e.timing(True)
        e.policy_step(state, eps=eps, action=act_, logp=lp, value=val, mean=mu)
        torch.cuda.synchronize()
        kernels = e.timing_kernels()
        e.timing(False)
        assert ("wide_policy_fused_kernel" in kernels) == (mode == "fused"), kernels
        outs[mode] = [x.cpu() for x in (act_, lp, val, mu)]
        std = eng.networks["actor"].actor_logstd.detach().exp().cpu()
        assert torch.equal(outs[mode][0], eps.cpu() * std + outs[mode][3])
    (a_f, lp_f, v_f, m_f), (a_l, lp_l, v_l, m_l) = outs["fused"], outs["layered"]
    for name, x, y in (("mean", m_f, m_l), ("value", v_f, v_l)):
        err = float((x - y).abs().max()) / (float(y.abs().max()) + 1e-12)
        print(f"fused vs layered rollout {name}: max err {err:.3e} of scale, "
              f"bitwise {torch.equal(x, y)}")
        assert err <= 1e-6, (name, err)
    torch.testing.assert_close(lp_f, lp_l, rtol=1e-5, atol=1e-5)


def test_fused_kernels_bitwise_deterministic(gpu):
    """The fused bf16 kernels reduce in a fixed order: repeating a call on the same inputs gives
    bit-identical outputs (rollout policy step and minibatch gradient at the bench shapes)."""
    n, t, b = 4096, 16, 65536 // 4
    run, eng, ref, cfg = _agents(gpu, 11, num_envs=n, hidden=(256, 256), batch_size=b,
                                 precision="bf16")
    e = eng.engine
    g = torch.Generator().manual_seed(3)
    win0 = torch.randn(n, 17, 1, generator=g, dtype=torch.float64).to(gpu)
    obs = torch.randn(n, 17, generator=g, dtype=torch.float64).to(gpu)
    eps = torch.randn(n, 6, generator=g).to(gpu)
    e.pack_weights()
    outs = []
    for _ in range(6):
        win = win0.clone()
        st = torch.empty(n, 17, device=gpu)
        a, lp, v, mu = (torch.empty(n, 6, device=gpu), torch.empty(n, device=gpu),
                        torch.empty(n, device=gpu), torch.empty(n, 6, device=gpu))
        e.observe_act(win, st, obs=obs, eps=eps, action=a, logp=lp, value=v, mean=mu)
        outs.append(torch.cat([st.flatten(), a.flatten(), lp, v, mu.flatten(), win.flatten().float()]))
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), int((o != outs[0]).sum())
    rows_total = n * t
    states = torch.randn(rows_total, 17, generator=g).to(gpu)
    actions = torch.randn(rows_total, 6, generator=g).to(gpu)
    old_lp = torch.randn(rows_total, generator=g).to(gpu) - 5
    adv = torch.randn(rows_total, generator=g).to(gpu)
    vt = torch.randn(rows_total, generator=g).to(gpu)
    rows = torch.randperm(rows_total, generator=g)[:b].to(torch.int32).to(gpu)
    grads = []
    for _ in range(4):
        grad = torch.empty(e.n_params, device=gpu)
        loss = torch.empty(2, device=gpu)
        e.minibatch_grad(states, actions, old_lp, adv, vt, rows, b, grad, loss, 0.9, 1.1, 1e-4,
                         1.0 / b, 1.0 / (b * 6))
        grads.append(torch.cat([grad, loss]))
    for gr in grads[1:]:
        assert torch.equal(gr, grads[0]), int((gr != grads[0]).sum())


@pytest.mark.parametrize("n,t,f64_reward,with_done", [(512, 16, True, False),
                                                      (100, 37, False, True),
                                                      (96, 200, True, True),
                                                      (40, 300, True, False)])
def test_gae_stage_records_matches_two_pass(gpu, n, t, f64_reward, with_done):
    """ppo_gae_stage_records (the GAE scan with the record pass fused in) == ppo_gae followed by
    ppo_stage_records, byte for byte: adv / vtarget compared directly, the records through
    ppo_minibatch_grad_staged over minibatches covering every row (a record that differed in any
    field would move the gradient).  Ragged N (not a multiple of the 16-env block), T not a
    multiple of the 16-row chunk, the 16-chunk variant (T = 200) and the two-pass fallback
    (T > 256); terminations mid-trajectory."""
    from mujoco_reinforcement_learning_amd import engine as E
    b = 2048
    run, eng, ref, cfg = _agents(gpu, 13, num_envs=n, hidden=(256, 256), batch_size=b,
                                 precision="bf16")
    e = eng.engine
    assert e.fused
    g = torch.Generator().manual_seed(5)
    values = torch.randn(t + 1, n, generator=g).to(gpu)
    rdt = torch.float64 if f64_reward else torch.float32
    reward = torch.randn(t, n, generator=g, dtype=rdt).to(gpu)
    term = (torch.rand(t, n, generator=g) < 0.03).to(gpu)
    done = (term.cpu() | (torch.rand(t, n, generator=g) < 0.02)).to(gpu) if with_done else None
    states = torch.randn(t + 1, n, 17, generator=g).to(gpu)
    actions = torch.randn(t, n, 6, generator=g).to(gpu)
    old_lp = torch.randn(t, n, generator=g).to(gpu) - 5
    adv0, vt0 = torch.empty(t, n, device=gpu), torch.empty(t, n, device=gpu)
    adv1, vt1 = torch.full((t, n), float("nan"), device=gpu), torch.full((t, n), float("nan"), device=gpu)
    E.gae(values[:t], values[1:], reward, term, 0.99, 0.95, adv0, vt0, done=done)
    e.pack_weights()
    args = (0.9, 1.1, 1e-4, 1.0 / b, 1.0 / (b * 6))
    perm = torch.randperm(n * t, generator=g).to(torch.int32).to(gpu)
    chunks = [perm[i:i + b] for i in range(0, n * t, b)]

    def grads():
        out = []
        for rows in chunks:
            gr, lo = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
            e.minibatch_grad_staged(rows, rows.numel(), gr, lo, *args)
            out.append(torch.cat([gr, lo]))
        return out

    e.stage_records(states, actions, old_lp, adv0, vt0)
    ref_grads = grads()
    e.gae_stage_records(values[:t], values[1:], reward, term, 0.99, 0.95, adv1, vt1, states,
                        actions, old_lp, done=done)
    got = grads()
    torch.cuda.synchronize()
    assert torch.equal(adv0, adv1) and torch.equal(vt0, vt1)
    for a, c in zip(ref_grads, got):
        assert torch.equal(a, c), int((a != c).sum())


@pytest.mark.parametrize("with_count", [False, True])
def test_staged_records_and_adam_pack_match_unstaged(gpu, with_count):
    """ppo_stage_records + ppo_minibatch_grad_staged give the gradient and losses of
    ppo_minibatch_grad bit for bit (also with a device row count, the exact-DP shard form); and
    ppo_adam_pack updates p/m/v exactly like ppo_adam while leaving weight images that equal a
    fresh ppo_pack_weights (the next staged gradient with weights_current=True is identical to
    one that refreshes the images)."""
    from mujoco_reinforcement_learning_amd import engine as E
    n, t, b = 512, 16, 2048
    run, eng, ref, cfg = _agents(gpu, 12, num_envs=n, hidden=(256, 256), batch_size=b,
                                 precision="bf16")
    e = eng.engine
    assert e.fused
    g = torch.Generator().manual_seed(4)
    rows_total = n * t
    states = torch.randn(t + 1, n, 17, generator=g).to(gpu)  # buffer layout with slot T
    actions = torch.randn(t, n, 6, generator=g).to(gpu)
    old_lp = torch.randn(t, n, generator=g).to(gpu) - 5
    adv = torch.randn(t, n, generator=g).to(gpu)
    vt = torch.randn(t, n, generator=g).to(gpu)
    rows = torch.randperm(rows_total, generator=g)[:b].to(torch.int32).to(gpu)
    count = torch.tensor([b - 300], dtype=torch.int32, device=gpu) if with_count else None
    args = (0.9, 1.1, 1e-4, 1.0 / b, 1.0 / (b * 6))
    e.pack_weights()
    g0, l0 = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
    e.minibatch_grad(states, actions, old_lp, adv, vt, rows, b, g0, l0, *args, count=count)
    e.stage_records(states, actions, old_lp, adv, vt)
    g1, l1 = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
    e.minibatch_grad_staged(rows, b, g1, l1, *args, count=count)
    torch.cuda.synchronize()
    assert torch.equal(g0, g1), int((g0 != g1).sum())
    assert torch.equal(l0, l1)
    # Adam: pack variant vs plain kernel on copies of the same state
    p0 = eng.flat_params.clone()
    m = torch.rand(e.n_params, generator=g).to(gpu) * 1e-3
    v = torch.rand(e.n_params, generator=g).to(gpu) * 1e-6
    m2, v2 = m.clone(), v.clone()
    sc = (-1e-3, -2e-3, 0.3, 0.1, 0.999, 0.001, 1e-8)
    E.adam(p0, g1, m, v, e.n_actor, sc[0], sc[1], sc[3], sc[4], sc[5], sc[2], sc[6])
    e.adam_pack(g1, m2, v2, None, *sc)
    torch.cuda.synchronize()
    assert torch.equal(p0, eng.flat_params)
    assert torch.equal(m, m2) and torch.equal(v, v2)
    # device-schedule variant on the next step
    sched = torch.tensor([sc[0], sc[1], sc[2]], device=gpu)
    p1 = eng.flat_params.clone()
    E.adam(p1, g1, m, v, e.n_actor, sc[0], sc[1], sc[3], sc[4], sc[5], sc[2], sc[6])
    e.adam_pack(g1, m2, v2, sched, one_minus_beta1=sc[3], beta2=sc[4], one_minus_beta2=sc[5],
                eps=sc[6])
    torch.cuda.synchronize()
    assert torch.equal(p1, eng.flat_params)
    # images left by adam_pack == a fresh refresh
    g2, l2 = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
    e.minibatch_grad_staged(rows, b, g2, l2, *args, count=count, weights_current=True)
    g3, l3 = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
    e.minibatch_grad_staged(rows, b, g3, l3, *args, count=count, weights_current=False)
    torch.cuda.synchronize()
    assert torch.equal(g2, g3), int((g2 != g3).sum())
    assert torch.equal(l2, l3)
    assert not torch.equal(g2, g1)  # the parameters did move


def test_update_step_staged_matches_grad_plus_adam_pack(gpu):
    """ppo_update_step_staged (fused forward/backward + one tail launch: slab reduction, Adam,
    weight images, next-minibatch gather) gives bit-identical gradient, losses, p, m and v to
    ppo_minibatch_grad_staged + ppo_adam_pack, for two chained steps (the second consuming the
    rows and weight images the first left behind) and with host or device Adam scalars."""
    n, t, b = 512, 16, 2048
    run, eng, ref, cfg = _agents(gpu, 13, num_envs=n, hidden=(256, 256), batch_size=b,
                                 precision="bf16")
    e = eng.engine
    g = torch.Generator().manual_seed(5)
    rows_total = n * t
    states = torch.randn(t + 1, n, 17, generator=g).to(gpu)
    actions = torch.randn(t, n, 6, generator=g).to(gpu)
    old_lp = torch.randn(t, n, generator=g).to(gpu) - 5
    adv = torch.randn(t, n, generator=g).to(gpu)
    vt = torch.randn(t, n, generator=g).to(gpu)
    rows = [torch.randperm(rows_total, generator=g)[:b].to(torch.int32).to(gpu) for _ in range(2)]
    args = (0.9, 1.1, 1e-4, 1.0 / b, 1.0 / (b * 6))
    sc = [(-1e-3, -2e-3, 0.3), (-1.5e-3, -2.5e-3, 0.4)]
    hyper = dict(one_minus_beta1=0.1, beta2=0.999, one_minus_beta2=0.001, eps=1e-8)
    p0 = eng.flat_params.clone()
    m0 = torch.rand(e.n_params, generator=g).to(gpu) * 1e-3
    v0 = torch.rand(e.n_params, generator=g).to(gpu) * 1e-6
    e.stage_records(states, actions, old_lp, adv, vt)
    outs = {}
    for mode in ("separate", "fused_host", "fused_sched"):
        eng.flat_params.copy_(p0)
        m, v = m0.clone(), v0.clone()
        e.pack_weights()
        grads, losses = [], []
        for k in range(2):
            grad, loss = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
            s = dict(zip(("neg_step_actor", "neg_step_critic", "bc2_sqrt"), sc[k]), **hyper)
            if mode == "separate":
                e.minibatch_grad_staged(rows[k], b, grad, loss, *args, weights_current=k > 0)
                e.adam_pack(grad, m, v, None, **s)
            else:
                sched = torch.tensor(sc[k], device=gpu) if mode == "fused_sched" else None
                if sched is not None:
                    s = dict(hyper)
                e.update_step_staged(rows[k], b, grad, loss, m, v, *args, sched=sched,
                                     next_rows=rows[1] if k == 0 else None,
                                     weights_current=k > 0, rows_gathered=k > 0, **s)
            grads.append(grad.clone())
            losses.append(loss.clone())
        torch.cuda.synchronize()
        outs[mode] = (torch.cat(grads), torch.cat(losses), eng.flat_params.clone(), m, v)
    for mode in ("fused_host", "fused_sched"):
        for name, x, y in zip(("grad", "loss", "params", "m", "v"), outs["separate"], outs[mode]):
            assert torch.equal(x, y), (mode, name, int((x != y).sum()))
    assert not torch.equal(outs["separate"][2], p0)


@pytest.mark.parametrize("with_count", [False, True])
def test_fused_direct_records_match_gathered_copy(gpu, with_count):
    """ppo_ctx_fused_direct: the 8-wave fused kernel reading each row's staged record through the
    row indices (default) gives the gradient, losses and Adam state of the gathered-copy path bit
    for bit -- two chained ppo_update_step_staged steps (the second with rows_gathered, i.e. the
    rows the first step's tail gathered in copy mode) and ppo_minibatch_grad_staged with a device
    row count; minibatch sizes that are not a multiple of the 64-row chunk, and out-of-range rows
    (masked to zero as the prep gather does)."""
    n, t, b = 512, 16, 2000
    run, eng, ref, cfg = _agents(gpu, 14, num_envs=n, hidden=(256, 256), batch_size=b,
                                 precision="bf16")
    e = eng.engine
    assert e.fused and e.fused_direct()
    g = torch.Generator().manual_seed(6)
    rows_total = n * t
    states = torch.randn(t + 1, n, 17, generator=g).to(gpu)
    actions = torch.randn(t, n, 6, generator=g).to(gpu)
    old_lp = torch.randn(t, n, generator=g).to(gpu) - 5
    adv = torch.randn(t, n, generator=g).to(gpu)
    vt = torch.randn(t, n, generator=g).to(gpu)
    rows = [torch.randperm(rows_total, generator=g)[:b].to(torch.int32) for _ in range(2)]
    rows[1][7] = rows_total + 5  # out of range: a zero row in both modes
    rows = [r.to(gpu) for r in rows]
    count = torch.tensor([b - 333], dtype=torch.int32, device=gpu) if with_count else None
    args = (0.9, 1.1, 1e-4, 1.0 / b, 1.0 / (b * 6))
    hyper = dict(one_minus_beta1=0.1, beta2=0.999, one_minus_beta2=0.001, eps=1e-8)
    p0 = eng.flat_params.clone()
    m0 = torch.rand(e.n_params, generator=g).to(gpu) * 1e-3
    v0 = torch.rand(e.n_params, generator=g).to(gpu) * 1e-6
    e.stage_records(states, actions, old_lp, adv, vt)
    outs = {}
    for direct in (True, False):
        e.fused_direct(direct)
        assert e.fused_direct() == direct
        eng.flat_params.copy_(p0)
        m, v = m0.clone(), v0.clone()
        e.pack_weights()
        res = []
        for k in range(2):
            grad, loss = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
            e.update_step_staged(rows[k], b, grad, loss, m, v, *args, neg_step_actor=-1e-3,
                                 neg_step_critic=-2e-3, bc2_sqrt=0.3,
                                 next_rows=rows[1] if k == 0 else None,
                                 weights_current=k > 0, rows_gathered=k > 0, **hyper)
            res += [grad.clone(), loss.clone()]
        gc, lc = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
        e.minibatch_grad_staged(rows[1], b, gc, lc, *args, count=count, weights_current=True)
        torch.cuda.synchronize()
        outs[direct] = res + [gc, lc, eng.flat_params.clone(), m, v]
    e.fused_direct(True)
    for i, (x, y) in enumerate(zip(outs[True], outs[False])):
        assert torch.equal(x, y), (i, int((x != y).sum()))


@pytest.mark.parametrize("sched", [1])
@pytest.mark.parametrize("n,t,b", [(512, 16, 2000), (4096, 32, 65536)])
def test_fused_schedules_bitwise(gpu, monkeypatch, sched, n, t, b):
    """PPO_FUSED_SCHED (fused_body SCHED, round 6): the ReLU kernel with dW0 deferred into the next
    chunk's L1 pass (1) and also the head dW inside the dW1 pass (3) moves wave-local work between
    phases only -- gradient, losses and the Adam step are bitwise those of schedule 0, from one
    chunk per workgroup (b = 2000, a partial last chunk) to the headline's eight (b = 65,536)."""
    run, eng, ref, cfg = _agents(gpu, 15, num_envs=n, hidden=(256, 256), batch_size=b,
                                 precision="bf16")
    e = eng.engine
    assert e.fused
    g = torch.Generator().manual_seed(9)
    states = torch.randn(t + 1, n, 17, generator=g).to(gpu)
    actions = torch.randn(t, n, 6, generator=g).to(gpu)
    old_lp = torch.randn(t, n, generator=g).to(gpu) - 5
    adv = torch.randn(t, n, generator=g).to(gpu)
    vt = torch.randn(t, n, generator=g).to(gpu)
    rows = [torch.randperm(n * t, generator=g)[:b].to(torch.int32).to(gpu) for _ in range(2)]
    args = (0.9, 1.1, 1e-4, 1.0 / b, 1.0 / (b * 6))
    hyper = dict(one_minus_beta1=0.1, beta2=0.999, one_minus_beta2=0.001, eps=1e-8)
    p0 = eng.flat_params.clone()
    m0 = torch.rand(e.n_params, generator=g).to(gpu) * 1e-3
    v0 = torch.rand(e.n_params, generator=g).to(gpu) * 1e-6
    e.stage_records(states, actions, old_lp, adv, vt)
    outs = {}
    for s in (0, sched):
        monkeypatch.setenv("PPO_FUSED_SCHED", str(s))
        eng.flat_params.copy_(p0)
        m, v = m0.clone(), v0.clone()
        e.pack_weights()
        res = []
        for k in range(2):
            grad, loss = torch.empty(e.n_params, device=gpu), torch.empty(2, device=gpu)
            e.update_step_staged(rows[k], b, grad, loss, m, v, *args, neg_step_actor=-1e-3,
                                 neg_step_critic=-2e-3, bc2_sqrt=0.3,
                                 next_rows=rows[1] if k == 0 else None,
                                 weights_current=k > 0, rows_gathered=k > 0, **hyper)
            res += [grad.clone(), loss.clone()]
        torch.cuda.synchronize()
        outs[s] = res + [eng.flat_params.clone(), m, v]
    assert bool(torch.isfinite(outs[0][0]).all()) and float(outs[0][0].abs().max()) > 0
    for i, (x, y) in enumerate(zip(outs[0], outs[sched])):
        assert torch.equal(x, y), (sched, i, int((x != y).sum()))
