"""GPU: the evaluation rollout (Algorithm.test, base_algorithm.py:21-48) and the test-phase action
of PPOAgent.act (agent.py:35-38 / ppo_agent.py:36-38) against the oracle.

Bars: the flattened test-phase action equals the oracle's mean within f32 summation order (rtol
1e-5); the 1000-step evaluation mean reward within rtol 1e-5 (the rewards are f64 functions of
the f32 mean actions), the termination/reset pattern identical, the final observation window
within 1e-5.
"""
import pytest
import torch

from oracle import ppo_ref as R
from parity_util import make_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,window", [(1, 1), (37, 1), (8, 3)])
def test_act_test_phase_flattens_means(gpu, n, window):
    algo, agent, ref, env, cfg = make_pair(gpu, n=n, t=4, b=n, window=window)
    g = torch.Generator().manual_seed(n)
    state = torch.randn(n, window, 17, generator=g)
    torch.manual_seed(0)
    action, dist = agent.act(state.to(gpu), return_dist=True, test_phase=True)
    rng_after = torch.rand(3)
    torch.manual_seed(0)
    ref_action, ref_dist = ref.act(state, return_dist=True, test_phase=True)
    assert torch.equal(torch.rand(3), rng_after), "test phase must not draw from the generator"
    assert action.shape == (n * 6,) and ref_action.shape == (n * 6,)
    torch.testing.assert_close(action.cpu(), ref_action, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dist.mean.cpu(), ref_dist.mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dist.stddev.cpu(), ref_dist.stddev)


@pytest.mark.parametrize("p_term,window,steps", [(0.0, 1, 1000), (0.1, 3, 1000), (0.3, 1, 257)])
def test_eval_rollout_matches_oracle(gpu, p_term, window, steps):
    algo, agent, ref, env, cfg = make_pair(gpu, n=8, t=16, b=32, window=window, p_term=p_term,
                                           hidden=(64, 64))
    got = algo.test(visualize=False, steps=steps)
    exp = R.test(env, ref, steps=steps)
    assert isinstance(got, float)
    assert abs(got - exp) <= 1e-5 * abs(exp) + 1e-9, (got, exp)
    # the device step counter followed the oracle's (termination resets included)
    assert int(algo.environment_helper._test_step) == env.test_t
    win = algo.environment_helper.test_timestep.observation.cpu()
    torch.testing.assert_close(win, env.test_window, rtol=1e-5, atol=1e-5)
    assert agent.networks.training, "test() restores train mode (base_algorithm.py:47)"


def test_eval_rollout_after_training_iteration(gpu):
    """test() between iterations, as Algorithm.iterate does (base_algorithm.py:63-66): the
    evaluation reads the parameters the update just wrote."""
    algo, agent, ref, env, cfg = make_pair(gpu, n=16, t=16, b=64, epochs=1, p_term=0.05)
    torch.manual_seed(3)
    mem = algo.rollout()
    algo.calculate_advantages(mem)
    algo.train(mem)
    torch.manual_seed(3)
    ref_mem = R.rollout(env, ref)
    R.calculate_advantages(ref_mem, cfg)
    R.train(ref, ref_mem, 0)
    got = algo.test(steps=300)
    exp = R.test(env, ref, steps=300)
    assert abs(got - exp) <= 1e-5 * abs(exp) + 1e-9, (got, exp)
