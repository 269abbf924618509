"""Write an ENGINE checkpoint fixture (run on the GPU box; the result is committed under
tests/golden/engine_ckpt/ and read by tests/test_checkpoint_interop.py on the CPU).

The agent is the reference's own network layout at W=1 -- actor 2x64 ReLU with tanh head,
critic the hard-coded [128, 128] of models/critic.py:14 -- trained for one PPO iteration on the
engine, then saved with PPOEngineAgent.save() (agent.py:47-56 layout: networks/<ep>/networks.pth,
optimizer_actor.pth, optimizer_critic.pth, configurations.json).  probe.npz records what the
reference modules must reproduce after loading those files:
  x (32, 1, 17)          a fixed input
  mean, std, value       the engine's HIP forward on x
  grad                   a fixed gradient (parameters() order, actor then critic)
  params_after           the engine's parameters after one more Adam step (both optimizers)
                         with that gradient, starting from the saved state

usage: python tools/make_engine_ckpt.py OUT_DIR
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    out = os.path.abspath(sys.argv[1])
    dev = torch.device("cuda", 0)
    n, t, b = 16, 16, 64
    run = make_run(num_envs=n, horizon=t, hidden=(64, 64), critic_hidden="reference",
                   batch_size=b, epochs=2, rng="torch", experiment_path=out)
    torch.manual_seed(0)
    agent = PPOEngineAgent(run, device=dev)
    streams = make_synthetic_streams(n, t, 17, seed=3, p_terminate=0.05)
    algo = PPOEngine(SyntheticVecEnvHelper(streams, run, device=dev), agent, log=lambda m: None)
    torch.manual_seed(1)
    algo._iterate()
    run.dynamic_config.current_episode = 1
    agent.save()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(32, 1, 17, generator=g)
    with torch.no_grad():
        mean, std = agent.networks["actor"](x.to(dev))
        value = agent.get_state_value(x.to(dev))
    grad = torch.randn(agent.packed_params().numel(), generator=g) * 1e-2
    # scatter the packed gradient into the engine's padded flat layout, then one step of each
    # optimizer (FlatAdam.step -> ppo_adam), as ppo.py:122,135 do
    agent.flat_grad.zero_()
    base, off = agent.flat_params.data_ptr(), 0
    for p in agent.networks.parameters():
        o = (p.data_ptr() - base) // 4
        agent.flat_grad[o:o + p.numel()] = grad[off:off + p.numel()].to(dev)
        off += p.numel()
    agent.optimizers["critic"].step()
    agent.optimizers["actor"].step()
    torch.cuda.synchronize()
    np.savez(os.path.join(out, "probe.npz"), x=x.numpy(), mean=mean.cpu().numpy(),
             std=std.cpu().numpy(), value=value.cpu().numpy(), grad=grad.numpy(),
             params_after=agent.packed_params().cpu().numpy(), episode=np.array(1))
    print("wrote", out)


if __name__ == "__main__":
    main()
