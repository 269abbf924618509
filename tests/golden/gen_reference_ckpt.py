"""Generate tests/golden/reference_ckpt/ -- a checkpoint written by the REFERENCE's own modules and
torch.optim.Adam in the reference Agent.save layout (agent.py:47-56), for the GPU test that loads
it into the engine (tests/test_gpu_checkpoint.py).

Run here (the container that has /root/reference), never on the GPU box:

    python tests/golden/gen_reference_ckpt.py

The networks are the reference's at W=1: models.linear.actor.Actor (2x64 ReLU, O=17, A=6) and
models.critic.Critic (its hard-coded [128, 128]), the optimizers the two Adams of
PPOAgent.initialize_networks (ppo_agent.py:15-22), stepped twice with seeded gradients so the
saved moments are non-trivial.  probe.npz records what the engine must reproduce after
PPOEngineAgent.load(): the forward (mean, std, value) on a fixed x, and the parameters after one
more step of both optimizers with a fixed gradient.  Only data is written; no source travels.
"""
import os
import shutil
import sys

import numpy as np
import torch

REF_SRC = "/root/reference/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_ckpt")
EPISODE = 4


def main():
    sys.path.insert(0, REF_SRC)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gen_golden import _make_run
    from models.critic import Critic
    from models.linear.actor import Actor
    from torch import nn

    _make_run(17, 1, 6, [64, 64], "ReLU")
    torch.manual_seed(11)
    nets = nn.ModuleDict()
    nets["actor"] = Actor()
    nets["critic"] = Critic()
    opts = {k: torch.optim.Adam(nets[k].parameters(), lr=1e-4) for k in ("actor", "critic")}
    g = torch.Generator().manual_seed(12)
    for _ in range(2):
        for k in ("critic", "actor"):
            for p in nets[k].parameters():
                p.grad = torch.randn(p.shape, generator=g) * 1e-2
            opts[k].step()
    if os.path.exists(OUT):
        shutil.rmtree(OUT)
    path = f"{OUT}/networks/{EPISODE}"
    os.makedirs(path)
    torch.save(nets.state_dict(), f"{path}/networks.pth")
    for k, o in opts.items():
        torch.save(o.state_dict(), f"{path}/optimizer_{k}.pth")
    x = torch.randn(32, 1, 17, generator=g)
    with torch.no_grad():
        mean, std = nets["actor"](x)
        value = nets["critic"](x)[:, 0, :]  # critic.py applies the MLP to the last dim: (N, 1, 1)
    grad = torch.randn(sum(p.numel() for p in nets.parameters()), generator=g) * 1e-2
    off = 0
    for p in nets.parameters():
        p.grad = grad[off:off + p.numel()].view(p.shape).clone()
        off += p.numel()
    opts["critic"].step()
    opts["actor"].step()
    after = torch.cat([p.detach().flatten() for p in nets.parameters()])
    np.savez(f"{OUT}/probe.npz", x=x.numpy(), mean=mean.numpy(), std=std.numpy(),
             value=value.numpy(), grad=grad.numpy(), params_after=after.numpy(),
             episode=np.array(EPISODE))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
