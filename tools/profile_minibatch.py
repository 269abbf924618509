"""Drive a few headline-shape PPO iterations or minibatch updates for rocprofv3.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python tools/profile_minibatch.py
    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- python tools/profile_minibatch.py --mode mb
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", choices=("iter", "mb"), default="iter")
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--hidden", default="256,256")
    a = p.parse_args()
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.algorithm import PPOEngine
    from mujoco_reinforcement_learning_amd.environments import (SyntheticVecEnvHelper,
                                                                make_synthetic_streams)
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    from mujoco_reinforcement_learning_amd import engine as E
    dev = torch.device("cuda", 0)
    hidden = tuple(int(h) for h in a.hidden.split(","))
    run = make_run(hidden=hidden, rng="philox", epochs=1 if a.mode == "mb" else 10)
    torch.manual_seed(0)
    agent = PPOEngineAgent(run, device=dev)
    helper = SyntheticVecEnvHelper(make_synthetic_streams(4096, 128, 17, device=dev), run,
                                   device=dev)
    algo = PPOEngine(helper, agent, log=lambda m: None)
    algo._iterate()  # warm
    torch.cuda.synchronize()
    if a.mode == "iter":
        for _ in range(a.reps):
            algo._iterate()
    else:
        buf = algo.buffer
        rows = torch.empty(65536, dtype=torch.int32, device=dev)
        loss = torch.empty(2, device=dev)
        for r in range(a.reps * 8):
            E.feistel_rows(1, r, 0, 65536, 4096, 128, rows)
            agent.engine.minibatch_grad(buf.states, buf.actions, buf.logp, buf.advantage,
                                        buf.value_target, rows, 65536, agent.flat_grad, loss,
                                        0.9, 1.1, 1e-4, 1 / 65536, 1 / (65536 * 6))
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
