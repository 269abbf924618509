"""Shared parity machinery for the GPU iteration tests: the engine and the oracle built on the same
seeds and synthetic streams, per-optimizer-step gradient capture on both sides, and the
post-update parameter bar of BASELINE.json's north_star ("post-update parameters within 1e-5 rtol").

The bar (``assert_params_match``):
  * every parameter element is within rtol 1e-5 of the oracle (atol 1e-5 * lr, i.e. 1e-5 of one
    Adam step, for elements the update leaves near zero -- biases start at exactly 0);
  * EXCEPT an explicitly counted set: elements whose oracle gradient at some optimizer step was
    below EPS_FLIP of its tensor's largest gradient.  Adam's step is ~lr * m / sqrt(v), which is
    scale-free, so for such a component the f32 summation-order difference between the GEMMs
    (MFMA vs CPU MKL) is a large RELATIVE error of g and can even flip the sign of the step
    (up to 2 * lr per step).  Those elements are bounded by 2 * lr * steps, their count is
    asserted to be a small fraction and printed, and so is the observed maximum everywhere.
Per-step gradients are also compared directly (relative to each tensor's max), which localises a
failure to the first step that diverges.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from oracle import ppo_ref as R

EPS_FLIP = 1e-3          # |g| < EPS_FLIP * max|g| of the tensor at some step -> sign-flip-prone
MAX_OUTSIDE_FRACTION = 1e-3  # flip-prone elements actually outside rtol: at most 0.1 % of all
SMALL_PARAM_STEPS = 100      # |p| < 100 * lr: a parameter the size of a few Adam steps


def make_pair(gpu, n=16, t=32, b=128, epochs=2, hidden=(64, 64), critic_hidden=None, obs=17,
              act=6, window=1, p_term=0.05, activation="relu", rng="torch", seed=0,
              feature_extractor="MLP", latent=256, extractor_layers=1, **kw):
    """(algo, agent, ref, env, cfg): engine drop-ins and the oracle on identical inputs.
    feature_extractor="LSTM": the BiLSTM actor / critic (lstm.LSTMEngineAgent vs
    oracle.lstm_ref.RefLSTMAgent; their MLPs use ``hidden``)."""
    from mujoco_reinforcement_learning_amd.agent import make_agent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    critic_hidden = tuple(critic_hidden or hidden)
    streams = make_synthetic_streams(n, t, obs, seed=seed + 5, p_terminate=p_term)
    run = make_run(num_envs=n, horizon=t, obs_dim=obs, act_dim=act, window=window, hidden=hidden,
                   critic_hidden=critic_hidden, activation=activation, batch_size=b,
                   epochs=epochs, rng=rng, seed=seed, feature_extractor=feature_extractor,
                   latent=latent, extractor_layers=extractor_layers, **kw)
    torch.manual_seed(seed)
    agent = make_agent(run, device=gpu)
    helper = SyntheticVecEnvHelper(streams, run, device=gpu)
    algo = PPOEngine(helper, agent, log=lambda m: None)
    cfg = R.RefConfig(num_envs=n, horizon=t, obs_dim=obs, act_dim=act, window=window,
                      actor_hidden=tuple(hidden), critic_hidden=critic_hidden,
                      activation=activation, batch_size=b, epochs=epochs,
                      normalize_advantage=kw.get("normalize_advantage", False),
                      normalize_rewards=kw.get("normalize_rewards", False))
    torch.manual_seed(seed)
    if feature_extractor == "LSTM":
        from oracle import lstm_ref
        ref = lstm_ref.RefLSTMAgent(cfg, latent, extractor_layers)
    else:
        ref = R.RefAgent(cfg)
    env = R.RefSyntheticEnv(streams["base_obs"], streams["base_reward"],
                            streams["base_terminated"], window, act)
    return algo, agent, ref, env, cfg


def capture_engine_grads(algo) -> List[torch.Tensor]:
    """Record the flat gradient of every optimizer step (parameters() order), at the point the
    engine hands it to the all-reduce (eager train loop: rng='torch')."""
    out: List[torch.Tensor] = []
    agent, dp = algo.agent, algo.dp
    orig = dp.allreduce_grad

    def hook(g):
        orig(g)
        out.append(agent.packed(g).detach().cpu().clone())

    dp.allreduce_grad = hook
    return out


def capture_oracle_grads(ref) -> List[torch.Tensor]:
    """Record the oracle's gradient per optimizer step: ppo.py steps the critic then the actor
    (ppo.py:120-135); each minibatch's record is actor then critic (the flat layout)."""
    out: List[torch.Tensor] = []
    pending = {}

    def wrap(name):
        opt = ref.optimizers[name]
        orig = opt.step

        def step(*a, **k):
            pending[name] = torch.cat([p.grad.detach().flatten().clone()
                                       for p in ref.networks[name].parameters()])
            if name == "actor":  # the second step of the minibatch
                out.append(torch.cat([pending["actor"], pending["critic"]]))
            return orig(*a, **k)

        opt.step = step

    wrap("critic")
    wrap("actor")
    return out


def tensor_slices(ref) -> List[tuple]:
    """(name, lo, hi) of every parameter tensor in the flat parameters() order."""
    out, off = [], 0
    for name, p in ref.networks.named_parameters():
        out.append((name, off, off + p.numel()))
        off += p.numel()
    return out


def compare_step_grads(g_eng: Sequence[torch.Tensor], g_ref: Sequence[torch.Tensor], ref,
                       rel: float, steps: Optional[int] = None) -> float:
    """Per-step gradients: max |g_eng - g_ref| <= rel * max|g_ref| per tensor, for the first
    ``steps`` steps (later steps see parameters that already differ by the flip-prone set).
    Returns the worst relative error seen."""
    assert len(g_eng) == len(g_ref), (len(g_eng), len(g_ref))
    worst = 0.0
    for k, (ge, gr) in enumerate(zip(g_eng, g_ref)):
        if steps is not None and k >= steps:
            break
        for name, lo, hi in tensor_slices(ref):
            scale = float(gr[lo:hi].abs().max()) + 1e-30
            err = float((ge[lo:hi] - gr[lo:hi]).abs().max()) / scale
            worst = max(worst, err)
            assert err <= rel, f"step {k} {name}: grad err {err:.3e} of max {scale:.3e}"
    return worst


def flip_prone(g_ref: Sequence[torch.Tensor], ref) -> torch.Tensor:
    """Elements whose oracle gradient was below EPS_FLIP of its tensor's max at some step."""
    mask = torch.zeros_like(g_ref[0], dtype=torch.bool)
    for gr in g_ref:
        for _, lo, hi in tensor_slices(ref):
            seg = gr[lo:hi].abs()
            mask[lo:hi] |= seg < EPS_FLIP * float(seg.max())
    return mask


def assert_params_match(p_eng: torch.Tensor, p_ref: torch.Tensor, g_ref: Sequence[torch.Tensor],
                        ref, lr: float, rtol: float = 1e-5, label: str = "",
                        max_outside: float = MAX_OUTSIDE_FRACTION) -> dict:
    """The north_star bar on post-update parameters (module docstring); returns the statistics
    it printed."""
    steps = len(g_ref)
    diff = (p_eng - p_ref).abs()
    tol = rtol * p_ref.abs() + rtol * lr
    prone = flip_prone(g_ref, ref)
    bad = (diff > tol) & ~prone
    stats = {"elements": diff.numel(), "steps": steps,
             "max_abs": float(diff.max()),
             "max_rel_nonprone": float((diff / (p_ref.abs() + lr))[~prone].max()),
             "flip_prone": int(prone.sum()),
             "flip_prone_outside_rtol": int(((diff > tol) & prone).sum()),
             "violations": int(bad.sum())}
    print(f"param parity {label}: {stats}")
    if bool(bad.any()):
        i = int(torch.nonzero(bad)[0])
        raise AssertionError(f"{label}: {int(bad.sum())} elements outside rtol {rtol} that are "
                             f"not flip-prone; first at {i}: engine {float(p_eng[i])!r} oracle "
                             f"{float(p_ref[i])!r} ({stats})")
    assert stats["flip_prone_outside_rtol"] <= max_outside * diff.numel(), stats
    assert stats["max_abs"] <= 2 * lr * steps, stats
    return stats


def run_iteration_pair(algo, agent, ref, env, cfg, seed_roll=1234, seed_train=99):
    """One rollout + GAE + train on both sides with the same torch RNG streams; returns
    (mem, ref_mem, engine step grads, oracle step grads)."""
    torch.manual_seed(seed_roll)
    mem = algo.rollout()
    algo.calculate_advantages(mem)
    torch.manual_seed(seed_roll)
    ref_mem = R.rollout(env, ref)
    R.calculate_advantages(ref_mem, cfg)
    g_eng = capture_engine_grads(algo)
    g_ref = capture_oracle_grads(ref)
    torch.manual_seed(seed_train)
    algo.train(mem)
    torch.manual_seed(seed_train)
    R.train(ref, ref_mem, 0)
    torch.cuda.synchronize()
    return mem, ref_mem, g_eng, g_ref


def own_gae(mem, cfg):
    """The oracle's GAE recomputed on the engine's own rollout tensors (bit-exact bar)."""
    rewards = mem["reward"].cpu()
    if cfg.normalize_rewards:
        rewards = rewards - rewards.mean(dim=1).unsqueeze(1)
        rewards = rewards / rewards.std(dim=1).unsqueeze(1)
    term = mem["terminated"].cpu().unsqueeze(-1)
    done = term.clone()
    done[:, -1] = True
    return R.generalized_advantage_estimate(cfg.gamma, cfg.lmbda, mem["current_state_value"].cpu(),
                                            mem["next_state_value"].cpu(), rewards, done, term)


# ------------------------------------------------------------------------------------------------
# Step-wise ("teacher-forced") parity: every optimizer step of the iteration, started from the
# ORACLE's own state at that step (parameters, Adam moments, step count) and the oracle's rollout
# buffer, must land on the oracle's post-step parameters.  A free-running multi-step comparison
# amplifies the f32 summation-order noise chaotically once any near-zero gradient component flips
# an Adam step (±lr); re-synchronising the state per step measures each step's arithmetic alone.
# ------------------------------------------------------------------------------------------------
def record_oracle_steps(ref) -> List[dict]:
    """Per minibatch: parameters / Adam moments / step count before, gradient, parameters after
    (actor then critic, parameters() order).  ppo.py steps the critic, then the actor."""
    out: List[dict] = []
    cur = {}

    def state_of(opt, params):
        ms, vs = [], []
        for p in params:
            st = opt.state.get(p, {})
            ms.append(st["exp_avg"].flatten().clone() if "exp_avg" in st else torch.zeros(p.numel()))
            vs.append(st["exp_avg_sq"].flatten().clone() if "exp_avg_sq" in st
                      else torch.zeros(p.numel()))
        k = int(float(opt.state[params[0]]["step"])) if params[0] in opt.state else 0
        return torch.cat(ms), torch.cat(vs), k

    def wrap(name):
        opt = ref.optimizers[name]
        orig = opt.step
        params = list(ref.networks[name].parameters())

        def step(*a, **kw):
            m, v, k = state_of(opt, params)
            cur[name] = {"p": torch.cat([p.detach().flatten().clone() for p in params]), "m": m,
                         "v": v, "k": k, "lr": opt.param_groups[0]["lr"],
                         "g": torch.cat([p.grad.detach().flatten().clone() for p in params])}
            r = orig(*a, **kw)
            cur[name]["p_after"] = torch.cat([p.detach().flatten().clone() for p in params])
            if name == "actor":
                rec = {key: torch.cat([cur["actor"][key], cur["critic"][key]])
                       for key in ("p", "m", "v", "g", "p_after")}
                rec["k"] = cur["actor"]["k"]
                rec["lr"] = cur["actor"]["lr"]
                assert cur["critic"]["k"] == rec["k"] and cur["critic"]["lr"] == rec["lr"]
                out.append(rec)
            return r

        opt.step = step

    wrap("critic")
    wrap("actor")
    return out


def replay_rows(seed_train: int, n: int, t: int, b: int, epochs: int, act: int) -> List[torch.Tensor]:
    """The reference's minibatch rows (ppo.py:101-108) for a train() seeded with seed_train:
    per epoch randperm(N*T), then per minibatch the (B, A) sample ppo.py:110 draws and drops.
    Returned as time-major storage rows t*N + n (int32) per optimizer step."""
    torch.manual_seed(seed_train)
    rows = []
    m = int(t * n / b)
    for _ in range(epochs):
        perm = torch.randperm(n * t)
        for i in range(m):
            torch.randn(b, act)
            f = perm[i * b:(i + 1) * b]
            rows.append(((f % t) * n + f // t).to(torch.int32))
    return rows


def _to_flat(agent, packed: torch.Tensor, flat: torch.Tensor) -> None:
    """Scatter a parameters()-order vector into the engine's padded flat layout."""
    base, off = agent.flat_params.data_ptr(), 0
    for p in agent.networks.parameters():
        o = (p.data_ptr() - base) // 4
        flat[o:o + p.numel()] = packed[off:off + p.numel()].to(flat.device)
        off += p.numel()


KINK_TAU = 1e-5  # |pre-activation| < KINK_TAU * (its row's largest): within f32 summation noise


class _KinkReLU(torch.autograd.Function):
    """ReLU whose derivative at near-kink inputs (|z| < KINK_TAU * row max) is forced to
    ``kink`` (0 or 1) instead of the sign of z: the two extremes an f32 evaluation can land on."""

    @staticmethod
    def forward(ctx, z, kink):
        near = z.abs() < KINK_TAU * z.abs().amax(dim=1, keepdim=True)
        ctx.save_for_backward(z, near)
        ctx.kink = kink
        return z.clamp_min(0)

    @staticmethod
    def backward(ctx, gy):
        z, near = ctx.saved_tensors
        d = (z > 0).to(gy.dtype)
        if ctx.kink is not None:
            d = torch.where(near, torch.full_like(d, float(ctx.kink)), d)
        return gy * d, None


def f64_step_grad(ref, cfg, ref_mem, p_packed: torch.Tensor, rows: torch.Tensor, kink=None):
    """The minibatch gradient of ppo.py:109-135 evaluated in float64 at the given parameters on
    the given storage rows (t*N + n): the arbiter when the engine and the f32 oracle disagree.
    kink = 0 / 1 forces the ReLU derivative at near-kink inputs (_KinkReLU).  Also returns, per
    Linear layer, the smallest |output|/row max (how close some ReLU input sits to its kink)."""
    import copy
    n, t = cfg.num_envs, cfg.horizon
    f = (rows.long() % n) * t + rows.long() // n  # storage row -> reference flat index n*T + t
    flat = {k: v.reshape(n * t, *v.shape[2:]) for k, v in ref_mem.items()}
    nets = copy.deepcopy(ref.networks).double()
    off = 0
    with torch.no_grad():
        for p in nets.parameters():
            p.copy_(p_packed[off:off + p.numel()].view(p.shape).double())
            off += p.numel()
    if cfg.activation == "relu":
        for blk in (nets["actor"].actor, nets["critic"].network):
            for i, m in enumerate(blk.first_layers):
                if isinstance(m, torch.nn.ReLU):
                    blk.first_layers[i] = _KinkModule(kink)
    x = flat["current_state"][f].double()
    kinks = []

    def hook(mod, inp, out):
        z = out.detach().abs()
        kinks.append(float((z / z.amax(dim=1, keepdim=True).clamp_min(1e-300)).min()))

    hs = [m.register_forward_hook(hook) for m in nets.modules() if isinstance(m, torch.nn.Linear)]
    mean, std = nets["actor"](x)
    dist = torch.distributions.Normal(mean, std)
    new_lp = dist.log_prob(flat["action"][f].double()).sum(dim=1)
    v = nets["critic"](x)
    lc = torch.nn.functional.huber_loss(v, flat["current_state_value_target"][f].double(),
                                        reduction="mean")
    ratio = (new_lp - flat["action_log_prob"][f].double()).exp()[:, None]
    adv = flat["advantage"][f].double()
    la = -torch.min(ratio * adv, torch.clamp(ratio, 1 - cfg.clip_epsilon, 1 + cfg.clip_epsilon)
                    * adv).mean() - dist.entropy().mean() * cfg.entropy_eps
    (la + lc).backward()
    for h in hs:
        h.remove()
    return torch.cat([p.grad.flatten() for p in nets.parameters()]), kinks


class _KinkModule(torch.nn.Module):
    def __init__(self, kink):
        super().__init__()
        self.kink = kink

    def forward(self, z):
        return _KinkReLU.apply(z, self.kink)


KINK_FRACTION_CAP = 0.15         # ReLU nets: gradient elements moved by kink flips, per step
ENGINE_KINK_FRACTION_CAP = 0.10  # ... of which the engine is off the float64 gradient, per step
# (observed at Humanoid 3x512 ReLU, B = 2048, 8 steps: up to 10.6 % and 6.3 % of the 1.45 M
# elements per step; the tanh net of the same shape has none -- test_iteration_humanoid_tanh_f32)


def stepwise_parity(algo, agent, ref, cfg, ref_mem, steps: List[dict], rows: List[torch.Tensor],
                    rtol: float = 1e-5, label: str = "", strict: bool = False) -> dict:
    """For every recorded oracle step k: load the oracle's (p, m, v, step count) into the engine,
    run ppo_minibatch_grad on the oracle's rollout buffer (time-major) with step k's rows, then the
    engine's Adam.  Bars: gradient within 2e-5 of each tensor's max; post-step parameters within
    rtol (atol rtol*lr) except two counted sets: tiny gradients (|g_oracle| < EPS_FLIP of the
    tensor's max at that step; bounded by 2*lr and MAX_OUTSIDE_FRACTION of the elements) and
    parameters the size of a few Adam steps (|p| < SMALL_PARAM_STEPS*lr; held to rtol 1e-3).
    Elements whose gradient differs by more than 1e-4 relative (ReLU kink flips, counted and
    bounded per tensor at the gradient check) are reported as kink_outside.  A gradient sign
    flip outside the tiny-gradient set fails.  The kink-moved elements are capped per step
    (KINK_FRACTION_CAP, ENGINE_KINK_FRACTION_CAP of all elements).

    strict=True (nets without kinks, e.g. tanh): no float64 arbitration and no kink / oracle-off
    exemptions -- every gradient element within 2e-5 of its tensor's max, every parameter within
    rtol except the counted tiny-gradient set and the parameters of the size of a few Adam steps
    (held to rtol 1e-3: for them rtol on p is rtol on one update, i.e. on the relative error of
    a gradient element, which f32 summation cancellation alone puts near 1e-4)."""
    dev = agent.device
    n, t = cfg.num_envs, cfg.horizon
    tm = lambda x: x.transpose(0, 1).reshape(t * n, *x.shape[2:]).contiguous().to(dev)
    states = tm(ref_mem["current_state"].reshape(n, t, -1))
    actions = tm(ref_mem["action"])
    old_lp = tm(ref_mem["action_log_prob"])
    adv = tm(ref_mem["advantage"][..., 0])
    vt = tm(ref_mem["current_state_value_target"][..., 0])
    b = cfg.batch_size
    eng = agent.engine
    grad = torch.empty(eng.n_params, device=dev)
    loss = torch.empty(2, device=dev)
    totals = {"steps": len(steps), "sign_flips": 0, "outside": 0, "grad_worst": 0.0,
              "max_rel": 0.0}
    for k, (rec, r) in enumerate(zip(steps, rows)):
        _to_flat(agent, rec["p"], agent.flat_params)
        agent.flat_m.zero_()
        agent.flat_v.zero_()
        _to_flat(agent, rec["m"], agent.flat_m)
        _to_flat(agent, rec["v"], agent.flat_v)
        for name in ("actor", "critic"):
            agent.optimizers[name].step_count = rec["k"]
            agent.optimizers[name].param_groups[0]["lr"] = rec["lr"]
        eng.minibatch_grad(states, actions, old_lp, adv, vt, r.to(dev), b, grad, loss,
                           1.0 - cfg.clip_epsilon, 1.0 + cfg.clip_epsilon, cfg.entropy_eps,
                           1.0 / b, 1.0 / (b * cfg.act_dim))
        agent.flat_grad.copy_(grad)
        g_eng = agent.packed(grad).cpu()
        g64 = None
        oracle_off = torch.zeros_like(g_eng, dtype=torch.bool)
        engine_off = torch.zeros_like(g_eng, dtype=torch.bool)  # near-kink-explained elements
        step_kinks = 0
        for name, lo, hi in tensor_slices(ref):
            gr, ge = rec["g"][lo:hi], g_eng[lo:hi]
            scale = float(gr.abs().max()) + 1e-30
            err = float((ge - gr).abs().max()) / scale
            l2 = float((ge - gr).norm() / (gr.norm() + 1e-30))
            # element-wise 2e-5 of the max except a counted few: a ReLU input whose f32
            # pre-activation sits within summation-order noise of 0 takes the other branch on one
            # side, moving that row's whole contribution to the unit's gradients
            n_off = int(((ge - gr).abs() > 2e-5 * scale).sum())
            totals["grad_worst"] = max(totals["grad_worst"], err)
            totals["grad_l2_worst"] = max(totals.get("grad_l2_worst", 0.0), l2)
            totals["kink_elements"] = totals.get("kink_elements", 0) + n_off
            step_kinks += n_off
            if strict:
                assert err <= 2e-5, f"{label} step {k} {name}: grad err {err:.3e} of max (strict)"
                continue
            if l2 <= 1e-4 and err <= 1e-2 and n_off <= max(4, 1e-4 * (hi - lo)):
                continue
            # disagreement beyond f32 noise: the float64 gradient decides which side is off; the
            # engine must be within 1e-5 (rel L2) of it, and the oracle's own off elements are
            # recorded so the parameter check below does not hold the engine to them
            if g64 is None:
                g64, kinks = f64_step_grad(ref, cfg, ref_mem, rec["p"], r)
            e_eng = float((ge.double() - g64[lo:hi]).norm() / g64[lo:hi].norm())
            e_ref = float((gr.double() - g64[lo:hi]).norm() / g64[lo:hi].norm())
            totals["f64_arbitrated"] = totals.get("f64_arbitrated", 0) + 1
            totals["f64_engine_worst"] = max(totals.get("f64_engine_worst", 0.0), e_eng)
            totals["f64_oracle_worst"] = max(totals.get("f64_oracle_worst", 0.0), e_ref)
            if e_eng > 1e-5:
                # the engine's f32 evaluation may have put a near-kink ReLU input (|z| within
                # KINK_TAU of its row's scale) on the other branch: its deviation from the exact
                # gradient must stay within the whole near-kink contribution |g(kink=1) - g(kink=0)|
                g1, _ = f64_step_grad(ref, cfg, ref_mem, rec["p"], r, kink=1)
                g0, _ = f64_step_grad(ref, cfg, ref_mem, rec["p"], r, kink=0)
                span = float((g1[lo:hi] - g0[lo:hi]).norm() / g64[lo:hi].norm())
                totals["kink_span_worst"] = max(totals.get("kink_span_worst", 0.0), span)
                assert e_eng <= span + 1e-5, (
                    f"{label} step {k} {name}: grad err {err:.3e} of max, rel L2 {l2:.3e}; vs "
                    f"float64: engine {e_eng:.3e}, f32 oracle {e_ref:.3e}, near-kink span "
                    f"{span:.3e}; min |pre-act|/row max per layer {kinks}")
                g64e = g64[lo:hi].float()
                engine_off[lo:hi] = (ge - g64e).abs() > 1e-4 * g64e.abs() + 2e-6 * float(g64e.abs().max())
            g64s = g64[lo:hi].float()
            oracle_off[lo:hi] = (gr - g64s).abs() > 1e-4 * g64s.abs() + 2e-6 * float(g64s.abs().max())
        n_el = g_eng.numel()
        totals["kink_fraction_worst"] = max(totals.get("kink_fraction_worst", 0.0), step_kinks / n_el)
        totals["engine_kink_fraction_worst"] = max(totals.get("engine_kink_fraction_worst", 0.0),
                                                   int(engine_off.sum()) / n_el)
        assert step_kinks <= KINK_FRACTION_CAP * n_el, (label, k, step_kinks, n_el)
        assert int(engine_off.sum()) <= ENGINE_KINK_FRACTION_CAP * n_el, (label, k, totals)
        agent.step_both()
        p_eng = agent.packed_params().cpu()
        diff = (p_eng - rec["p_after"]).abs()
        tol = rtol * rec["p_after"].abs() + rtol * rec["lr"]
        flip = torch.sign(g_eng) != torch.sign(rec["g"])
        small = torch.zeros_like(flip)
        for _, lo, hi in tensor_slices(ref):
            seg = rec["g"][lo:hi].abs()
            small[lo:hi] = seg < EPS_FLIP * float(seg.max())
        totals["engine_kink_elements"] = totals.get("engine_kink_elements", 0) + int(engine_off.sum())
        assert not bool((flip & ~small & ~oracle_off & ~engine_off).any()), \
            f"{label} step {k}: sign flip of a large gradient"
        # tiny-gradient elements: Adam's update lr*g/(|g|+eps) passes the RELATIVE error of such
        # a g (f32 summation order, cancellation) straight into the step, sign flips included;
        # they are counted and bounded by 2*lr, everything else must meet rtol
        outside = diff > tol
        # parameters of the size of a few Adam steps (zero-initialised biases / log-std): rtol on
        # p is rtol on one or two updates, i.e. on the relative error of g itself -> rtol 1e-3
        tiny_p = rec["p_after"].abs() < SMALL_PARAM_STEPS * rec["lr"]
        within = ~small & ~(tiny_p & (diff <= 1e-3 * rec["p_after"].abs() + rtol * rec["lr"]))
        # the gradient elements moved by a kink flip (counted above) move their Adam step too
        kink = (g_eng - rec["g"]).abs() > 1e-4 * rec["g"].abs()
        bad = outside & within & ~kink & ~oracle_off & ~engine_off
        totals["kink_outside"] = totals.get("kink_outside", 0) + int((outside & within & kink).sum())
        totals["oracle_off_outside"] = totals.get("oracle_off_outside", 0) + int(
            (outside & within & oracle_off).sum())
        totals["small_param_outside"] = totals.get("small_param_outside", 0) + int(
            (outside & ~small & tiny_p).sum())
        assert float(diff.max()) <= 2 * rec["lr"], (label, k, float(diff.max()))
        totals["sign_flips"] += int(flip.sum())
        totals["outside"] += int(outside.sum())
        totals["tiny_grad"] = totals.get("tiny_grad", 0) + int(small.sum())
        totals["max_rel"] = max(totals["max_rel"],
                                float((diff / (rec["p_after"].abs() + rec["lr"]))[~small].max()))
        if bool(bad.any()):
            i = int(torch.nonzero(bad)[0])
            raise AssertionError(f"{label} step {k}: {int(bad.sum())} params outside rtol {rtol} "
                                 f"with |g| >= {EPS_FLIP} of the tensor max; first {i}: engine "
                                 f"{float(p_eng[i])!r} oracle {float(rec['p_after'][i])!r} "
                                 f"g {float(g_eng[i])!r} vs {float(rec['g'][i])!r}")
        assert int((outside & ~oracle_off).sum()) <= MAX_OUTSIDE_FRACTION * diff.numel(), \
            (label, k, totals)
    print(f"stepwise parity {label}: {totals}")
    return totals


# ------------------------------------------------------------------------------------------------
# bf16 step-wise parity: the engine's bf16 kernels (precision "bf16") restarted at every optimizer
# step from the bf16-EMULATION oracle's own state and held to that step's gradient evaluated by the
# f64-accumulated emulation (the same bf16-rounded operands, sums without f32 rounding).  What is
# left is the engine's f32 summation order flipping a bf16 rounding of an intermediate (1 bf16 ulp
# = 2^-8 relative), which cascades through the layers; the fixed bars below sit at ~3x the
# emulation's own f32-vs-f64 spread at these shapes.
# ------------------------------------------------------------------------------------------------
WELL_DETERMINED = 1e-2  # bf16 step-wise: |g| >= 1e-2 of the tensor's max has a determined sign


def load_packed(nets, p_packed: torch.Tensor) -> None:
    """Copy a parameters()-order vector into a ModuleDict's parameters (any float dtype)."""
    off = 0
    with torch.no_grad():
        for p in nets.parameters():
            p.copy_(p_packed[off:off + p.numel()].view(p.shape).to(p.dtype))
            off += p.numel()


def bf16_f64_grad(ref0, mem, rows: torch.Tensor, cfg, p_packed=None, bf16_fn=None,
                  state_dtype=torch.float64) -> torch.Tensor:
    """The minibatch gradient of ppo.py:109-135 under the bf16 emulation accumulated in float64,
    at parameters ``p_packed`` (default: ``ref0``'s) on storage rows ``rows`` (t*N + n) of a
    reference-layout (N, T, ...) buffer ``mem``.  ``bf16_fn`` switches an agent to the emulation
    (oracle.ppo_ref.use_bf16_gemms, oracle.lstm_ref.use_bf16_gemms, oracle.cnn_ref.use_bf16);
    ``state_dtype`` None passes the stored states as they are (u8 pixel frames, whose scaling
    the caller routes to f64)."""
    import copy
    n, t = cfg.num_envs, cfg.horizon
    ref = copy.deepcopy(ref0)
    if p_packed is not None:
        load_packed(ref.networks, p_packed)
    (bf16_fn or R.use_bf16_gemms)(ref)
    ref.networks.to(torch.float64)
    r = rows.long()
    em = (r % n) * t + r // n  # storage row t*N + n -> the reference's env-major n*T + t
    flat = {k: mem[k].cpu().reshape(n * t, *mem[k].shape[2:]) for k in
            ("current_state", "action", "action_log_prob", "advantage",
             "current_state_value_target")}
    x = flat["current_state"][em]
    x = x.to(state_dtype) if state_dtype is not None else x
    _, dist = ref.act(x, return_dist=True)
    new_lp = dist.log_prob(flat["action"][em].double()).sum(dim=1)
    v = ref.get_state_value(x)
    vt = flat["current_state_value_target"][em].double().reshape(v.shape)
    lc = torch.nn.functional.huber_loss(v, vt, reduction="mean")
    ratio = (new_lp - flat["action_log_prob"][em].double().reshape(new_lp.shape)).exp()[:, None]
    a_ = flat["advantage"][em].double().reshape(ratio.shape)
    la = -torch.min(ratio * a_, torch.clamp(ratio, 1 - cfg.clip_epsilon, 1 + cfg.clip_epsilon)
                    * a_).mean() - dist.entropy().mean() * cfg.entropy_eps
    ref.networks.zero_grad()
    (la + lc).backward()
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).flatten()
                      for p in ref.networks.parameters()])


def grad_errors(g_eng: torch.Tensor, g64: torch.Tensor, ref) -> List[tuple]:
    """(name, max |err| / max |g64|, rel L2) per parameter tensor (all-zero tensors skipped)."""
    out = []
    for name, lo, hi in tensor_slices(ref):
        gr = g64[lo:hi]
        if float(gr.abs().max()) == 0.0:
            assert float(g_eng[lo:hi].abs().max()) == 0.0, name
            continue
        ge = g_eng[lo:hi].double()
        out.append((name, float((ge - gr).abs().max()) / float(gr.abs().max()),
                    float((ge - gr).norm() / gr.norm())))
    return out


def bf16_stepwise(agent, ref0, cfg, ref_mem, steps: List[dict], rows: List[torch.Tensor],
                  max_bar: float, l2_bar: float, update_bar: float, bf16_fn=None,
                  label: str = "", grad_fn=None) -> dict:
    """For every recorded step k of the bf16-emulation oracle (``steps``: record_oracle_steps,
    ``rows``: replay_rows): load the oracle's (p, m, v, step count, lr) into the engine, run the
    engine's bf16 minibatch gradient on the ORACLE's rollout buffer with step k's rows, then its
    Adam step.  Bars per tensor: the gradient against bf16_f64_grad at the same parameters within
    ``max_bar`` of the tensor's max and ``l2_bar`` relative L2; the parameter update (post - pre)
    against the oracle's own within ``update_bar`` relative L2 over the elements whose gradient
    sign is determined (|g| >= WELL_DETERMINED of the tensor's max), every element within 2*lr
    (Adam's step is scale-free: an element whose gradient is small against its tensor's max takes
    a full-size step whose sign follows the bf16 rounding noise).  Returns the observed maxima,
    beside the emulation's own f32-vs-f64 spread at the same states (rec["g"] is the
    f32-accumulated emulation's gradient)."""
    dev = agent.device
    n, t = cfg.num_envs, cfg.horizon
    tm = lambda x: x.transpose(0, 1).reshape(t * n, *x.shape[2:]).contiguous().to(dev)
    states = tm(ref_mem["current_state"].reshape(n, t, -1))
    actions = tm(ref_mem["action"])
    old_lp = tm(ref_mem["action_log_prob"])
    adv = tm(ref_mem["advantage"][..., 0])
    vt = tm(ref_mem["current_state_value_target"][..., 0])
    b = cfg.batch_size
    eng = agent.engine
    grad = torch.empty(eng.n_params, device=dev)
    loss = torch.empty(2, device=dev)
    obs = {"steps": len(steps), "grad_max": 0.0, "grad_l2": 0.0, "update_l2": 0.0,
           "param_max_abs_over_lr": 0.0}
    bad = []
    for k, (rec, r) in enumerate(zip(steps, rows)):
        _to_flat(agent, rec["p"], agent.flat_params)
        agent.flat_m.zero_()
        agent.flat_v.zero_()
        _to_flat(agent, rec["m"], agent.flat_m)
        _to_flat(agent, rec["v"], agent.flat_v)
        for name in ("actor", "critic"):
            agent.optimizers[name].step_count = rec["k"]
            agent.optimizers[name].param_groups[0]["lr"] = rec["lr"]
        if hasattr(eng, "pack_weights"):
            eng.pack_weights()
        eng.minibatch_grad(states, actions, old_lp, adv, vt, r.to(dev), b, grad, loss,
                           1.0 - cfg.clip_epsilon, 1.0 + cfg.clip_epsilon, cfg.entropy_eps,
                           1.0 / b, 1.0 / (b * cfg.act_dim))
        agent.flat_grad.copy_(grad)
        g_eng = agent.packed(grad).cpu()
        g64 = (grad_fn or bf16_f64_grad)(ref0, ref_mem, r, cfg, p_packed=rec["p"], bf16_fn=bf16_fn)
        own = {nm: (e, l) for nm, e, l in grad_errors(rec["g"], g64, ref0)}
        err_of = {}
        for name, err, l2 in grad_errors(g_eng, g64, ref0):
            err_of[name] = err
            obs["grad_max"] = max(obs["grad_max"], err)
            obs["grad_l2"] = max(obs["grad_l2"], l2)
            obs["emulation_spread_max"] = max(obs.get("emulation_spread_max", 0.0), own[name][0])
            obs["emulation_spread_l2"] = max(obs.get("emulation_spread_l2", 0.0), own[name][1])
            if err > max_bar or l2 > l2_bar:
                bad.append(("grad", k, name, err, l2, own[name]))
        agent.step_both()
        p_eng = agent.packed_params().cpu()
        obs["param_max_abs_over_lr"] = max(obs["param_max_abs_over_lr"],
                                           float((p_eng - rec["p_after"]).abs().max()) / rec["lr"])
        for name, lo, hi in tensor_slices(ref0):
            du_e = p_eng[lo:hi] - rec["p"][lo:hi]
            du_r = rec["p_after"][lo:hi] - rec["p"][lo:hi]
            # the update bar holds where the gradient's sign is determined (|g| >= WELL of the
            # tensor's max in the f64 emulation); the rest are counted, bounded by 2*lr above
            g = g64[lo:hi].abs()
            well = g >= max(WELL_DETERMINED, 3 * err_of.get(name, 0.0)) * float(g.max())
            obs["sign_free_elements"] = obs.get("sign_free_elements", 0) + int((~well).sum())
            if float(du_r[well].norm()) == 0.0:
                continue
            u = float((du_e[well] - du_r[well]).norm() / du_r[well].norm())
            obs["update_l2"] = max(obs["update_l2"], u)
            if u > update_bar:
                bad.append(("update", k, name, u))
    print(f"bf16 stepwise {label}: {obs}")
    assert not bad, (label, bad[:8])
    assert obs["param_max_abs_over_lr"] <= 2.0 + 1e-3, obs
    return obs
