"""ExponentialLRFacade against torch.optim.lr_scheduler.ExponentialLR (ppo_agent.py:19-22,
ppo.py:146-148): the same learning-rate sequence, bit for bit, and the same Adam step sizes
(FlatAdam.scalars restates adam.py's python-double math); state dicts load across.  CPU only:
the facades are host bookkeeping (no kernel runs)."""
import torch

from mujoco_reinforcement_learning_amd.agent import ExponentialLRFacade, FlatAdam


def _pair(lr=1e-4, gamma=0.999):
    flat = torch.zeros(4, 32)
    params = [torch.nn.Parameter(flat[0, :16].view(4, 4))]
    flat_adam = FlatAdam(params, flat[0], flat[1], flat[2], flat[3], 0, 32, lr)
    ref_p = [torch.nn.Parameter(torch.zeros(4, 4))]
    ref_opt = torch.optim.Adam(ref_p, lr=lr)
    return (flat_adam, ExponentialLRFacade(flat_adam, gamma), ref_opt,
            torch.optim.lr_scheduler.ExponentialLR(ref_opt, gamma=gamma))


def test_lr_sequence_is_bitwise_torch():
    opt, sched, ref_opt, ref_sched = _pair()
    for k in range(300):
        assert opt.lr == ref_opt.param_groups[0]["lr"], k
        assert sched.get_last_lr() == ref_sched.get_last_lr(), k
        ref_opt.step()  # torch warns when the scheduler steps before the optimizer
        sched.step()
        ref_sched.step()
    assert sched.last_epoch == ref_sched.last_epoch == 300


def test_adam_step_sizes_follow_the_schedule():
    """step_size = lr / (1 - beta1^k), bias_correction2_sqrt = sqrt(1 - beta2^k) in python double
    (adam.py _single_tensor_adam), with lr read after each scheduler step."""
    opt, sched, _, _ = _pair(lr=3e-4, gamma=0.99)
    beta1, beta2 = opt.param_groups[0]["betas"]
    for k in range(1, 50):
        neg, bc2 = opt.scalars(k)
        assert neg == -(opt.lr / (1 - beta1 ** k))
        assert bc2 == (1 - beta2 ** k) ** 0.5
        sched.step()


def test_state_dicts_load_across():
    opt, sched, ref_opt, ref_sched = _pair()
    for _ in range(7):
        ref_opt.step()
        ref_sched.step()
    sched.load_state_dict(ref_sched.state_dict())
    assert sched.last_epoch == 7 and sched.gamma == ref_sched.gamma
    for _ in range(5):
        sched.step()
    ref2 = torch.optim.lr_scheduler.ExponentialLR(torch.optim.Adam([torch.nn.Parameter(
        torch.zeros(1))], lr=1e-4), gamma=0.5)
    ref2.load_state_dict(sched.state_dict())
    assert ref2.last_epoch == 12 and ref2.gamma == sched.gamma
