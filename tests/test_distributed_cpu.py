"""CPU, world_size 2 over gloo: the data-parallel design of SURVEY.md s8(e).

* shard_range / DataParallel bookkeeping;
* the one exchange (all-reduce SUM of the flat gradient);
* exact-DP equivalence of the reference loss (oracle, torch autograd): every rank takes the rows of
  the GLOBAL minibatch that fall in its env shard and divides by the global B; the summed
  gradients equal the single-process gradient (up to summation order).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from mujoco_reinforcement_learning_amd.distributed import DataParallel, shard_range


def test_shard_range():
    assert shard_range(16, 2, 0) == (0, 8) and shard_range(16, 2, 1) == (8, 16)
    assert shard_range(4096 * 8, 8, 7) == (7 * 4096, 8 * 4096)
    with pytest.raises(ValueError):
        shard_range(10, 3, 0)


def test_single_process_dataparallel_is_identity():
    dp = DataParallel(mode="exact")
    g = torch.arange(5.0)
    dp.allreduce_grad(g)
    assert dp.world == 1 and not dp.active and torch.equal(g, torch.arange(5.0))
    assert dp.loss_scale(64) == 64 and dp.my_shard(8) == (0, 8)
    with pytest.raises(ValueError):
        DataParallel(mode="bogus")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _loss_grads(agent, states, actions, old_lp, adv, vt, idx, b_global):
    """ppo.py:109-135 losses over rows ``idx`` with the mean taken over ``b_global`` rows."""
    agent.networks.zero_grad()
    x = states[idx][:, None, :]
    _, dist = agent.act(x, return_dist=True)
    new_lp = dist.log_prob(actions[idx]).sum(dim=1)
    v = agent.get_state_value(x)[:, 0]
    d = v - vt[idx]
    ad = d.abs()
    lc = torch.where(ad < 1, 0.5 * d * d, ad - 0.5).sum() / b_global
    ratio = (new_lp - old_lp[idx]).exp()
    a = adv[idx]
    la = -torch.min(ratio * a, torch.clamp(ratio, 0.9, 1.1) * a).sum() / b_global
    ent = (dist.entropy().sum() / (b_global * dist.mean.shape[1])) * 1e-4
    (la - ent + lc).backward()
    return torch.cat([p.grad.flatten() for p in agent.networks.parameters()])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.ppo_ref import RefAgent, RefConfig
    dp = DataParallel(mode="exact")
    assert dp.world == world and dp.rank == rank
    # the exchange itself
    g = torch.full((7,), float(rank + 1))
    dp.allreduce_grad(g)
    assert torch.equal(g, torch.full((7,), float(sum(range(1, world + 1)))))
    # exact-DP gradient: global minibatch, rows filtered to this rank's envs, global B scaling
    n_glob, t, b = 16, 8, 64
    cfg = RefConfig(num_envs=n_glob, horizon=t, actor_hidden=(32, 32), critic_hidden=(32, 32))
    torch.manual_seed(0)
    agent = RefAgent(cfg)
    gen = torch.Generator().manual_seed(1)
    states = torch.randn(n_glob * t, 17, generator=gen)
    actions = torch.randn(n_glob * t, 6, generator=gen) * 0.3
    old_lp = torch.randn(n_glob * t, generator=gen) - 5
    adv = torch.randn(n_glob * t, generator=gen)
    vt = torch.randn(n_glob * t, generator=gen)
    perm = torch.randperm(n_glob * t, generator=gen)[:b]  # flat f = env*T + t (ppo.py:99)
    lo, hi = dp.my_shard(n_glob // world)
    env = perm // t
    mine = perm[(env >= lo) & (env < hi)]
    g_local = _loss_grads(agent, states, actions, old_lp, adv, vt, mine, b)
    dp.allreduce_grad(g_local)
    if rank == 0:
        g_full = _loss_grads(agent, states, actions, old_lp, adv, vt, perm, b)
        out.put(float((g_local - g_full).abs().max() / g_full.abs().max()))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_exact_data_parallel_gradient_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    rel = q.get(timeout=5)
    assert rel < 1e-5, rel


class _FakeComm:
    def __init__(self):
        self.retired = False

    def retire(self):
        self.retired = True


def _agree_worker(rank, world, port, case, out):
    """DataParallel.build_comm with injected pieces: whatever fails on ONE rank, every rank ends
    with the same outcome and none is left blocked in a collective."""
    from mujoco_reinforcement_learning_amd.distributed import NativeCommUnavailable
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    dp = DataParallel()
    made = []

    def make_id():
        if case == "id_fails":
            raise RuntimeError("no RCCL on rank 0")
        return bytes(range(128))

    def make_comm(uid, dev, w, r):
        assert uid == bytes(range(128)), "every rank holds rank 0's id"
        if case == "init_fails" and r == 1:
            raise RuntimeError("ncclCommInitRank failed")
        c = _FakeComm()
        made.append(c)
        return c

    loadable = (lambda: rank != 1) if case == "not_loadable" else (lambda: True)
    try:
        comm = dp.build_comm(torch.device("cpu"), make_id=make_id, make_comm=make_comm,
                             loadable=loadable)
        res = "ok"
        assert comm is made[0]
    except NativeCommUnavailable:
        res = "unavailable"
    # the ranks still pair their collectives afterwards
    g = torch.full((3,), float(rank + 1))
    dp.allreduce_grad(g)
    out.put((rank, res, [c.retired for c in made], float(g[0])))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("case,want", [("ok", "ok"), ("id_fails", "unavailable"),
                                       ("init_fails", "unavailable"),
                                       ("not_loadable", "unavailable")])
def test_native_comm_build_agreed_across_ranks(case, want):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert [r[1] for r in res] == [want, want], res
    assert all(r[3] == 3.0 for r in res), res  # the exchange after the decision pairs up
    if case == "init_fails":
        assert res[0][2] == [True], res  # rank 0 built one and retired it
    if case == "ok":
        assert res[0][2] == [False] and res[1][2] == [False]


def test_capture_agreed_single_rank():
    dp = DataParallel()
    assert dp.capture_agreed(lambda: None) is None
    with pytest.raises(RuntimeError):  # no native communicator: a capture error is an error
        dp.capture_agreed(lambda: (_ for _ in ()).throw(RuntimeError("boom")))
    c = dp.comm = _FakeComm()
    assert dp.capture_agreed(lambda: (_ for _ in ()).throw(RuntimeError("boom"))) == "boom"
    assert dp.comm is None and c.retired
