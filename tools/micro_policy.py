"""Fused rollout step (ppo_observe_act, bf16 2x256) kernel time vs N, and actor-only /
critic-only variants, from per-dispatch event timing."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    dev = torch.device("cuda", 0)
    for n in (512, 2048, 4096, 16384, 65536):
        run = make_run(num_envs=n, hidden=(256, 256), rng="philox", precision="bf16",
                       batch_size=min(n, 65536))
        torch.manual_seed(0)
        agent = PPOEngineAgent(run, device=dev)
        e = agent.engine
        e.pack_weights()
        win = torch.randn(n, 17, 1, device=dev, dtype=torch.float64)
        obs = torch.randn(n, 17, device=dev, dtype=torch.float64)
        st = torch.empty(n, 17, device=dev)
        a, lp, v = (torch.empty(n, 6, device=dev), torch.empty(n, device=dev),
                    torch.empty(n, device=dev))
        for label, kw in (("both", dict(action=a, logp=lp, value=v)), ("actor", dict(action=a, logp=lp)),
                          ("critic", dict(value=v))):
            e.observe_act(win, st, obs=obs, seed=1, offset=0, **kw)
            torch.cuda.synchronize()
            e.timing(True, capacity=4096)
            for i in range(50):
                e.observe_act(win, st, obs=obs, seed=1, offset=i, **kw)
            torch.cuda.synchronize()
            ks = e.timing_kernels()
            e.timing(False)
            for k, rec in ks.items():
                print(f"N={n:6d} {label:6s} {1e3 * rec['ms'] / rec['launches']:8.2f} us  {k}")


if __name__ == "__main__":
    main()
