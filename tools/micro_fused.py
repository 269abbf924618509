"""Headline-shape fused minibatch gradients (B=65536, 2x256 ReLU, A=6) in a loop, for PMC runs
(rocprofv3 --pmc ...) on the fused update kernel alone."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main(reps: int = 20):
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    from mujoco_reinforcement_learning_amd import engine as E
    dev = torch.device("cuda", 0)
    b, n, t = 65536, 4096, 128
    run = make_run(hidden=(256, 256), rng="philox", precision="bf16")
    torch.manual_seed(0)
    agent = PPOEngineAgent(run, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    states = torch.randn(n * t, 17, device=dev, generator=g)
    actions = torch.randn(n * t, 6, device=dev, generator=g)
    logp = torch.randn(n * t, device=dev, generator=g) - 5
    adv = torch.randn(n * t, device=dev, generator=g)
    vt = torch.randn(n * t, device=dev, generator=g)
    rows = torch.empty(b, dtype=torch.int32, device=dev)
    loss = torch.empty(2, device=dev)
    eng = agent.engine
    eng.stage_records(states, actions, logp, adv, vt)
    for rep in range(reps):
        E.feistel_rows(1, rep, 0, b, n, t, rows)
        eng.minibatch_grad_staged(rows, b, agent.flat_grad, loss, 0.9, 1.1, 1e-4, 1 / b,
                                  1 / (b * 6), weights_current=rep > 0)
    torch.cuda.synchronize()
    print("ok", float(loss[0]))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
