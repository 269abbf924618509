"""Per-phase cycles of the fused rollout step (ppo_observe_act, ReLU 2x256, A=6, N=4096) from the
stamped diagnostic instantiation: wave 0's s_memtime deltas per phase, averaged over workgroups,
for actor (y=0) and critic (y=1) workgroups; plus the spread of workgroup start times."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

PHASES = ["prologue: obs / param / eps loads issued (Philox noise when no eps is given)", "LDS images + raw window out",
          "per-(row, slice) f64 mean / std (lane-parallel butterflies)", "standardised states -> X image + state out",
          "L0 MFMA + act -> A1", "L1 MFMA pass (issue)", "act -> A2 image",
          "heads (tanh, sample, logp / value) + writes"]


def main():
    from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
    from mujoco_reinforcement_learning_amd.runconfig import make_run
    dev = torch.device("cuda", 0)
    n = 4096
    run = make_run(num_envs=n, hidden=(256, 256), rng="philox", precision="bf16")
    torch.manual_seed(0)
    agent = PPOEngineAgent(run, device=dev)
    e = agent.engine
    e.pack_weights()
    win = torch.randn(n, 17, 1, device=dev, dtype=torch.float64)
    obs = torch.randn(n, 17, device=dev, dtype=torch.float64)
    st = torch.empty(n, 17, device=dev)
    a, lp, v = torch.empty(n, 6, device=dev), torch.empty(n, device=dev), torch.empty(n, device=dev)
    eps = torch.randn(n, 6, device=dev)
    for rep in range(3):
        e.phase_stamps(True)
        # the bench's form: the rollout's noise drawn ahead of the steps (eps given)
        e.observe_act(win, st, obs=obs, eps=eps, seed=1, offset=rep, action=a, logp=lp, value=v)
        # the policy kernel writes 11 slots per workgroup (phase_stamps views them as 13)
        s = e.phase_stamps(False).flatten()[:2 * 128 * 11].view(2, 128, 11).double()
    g = n // 32  # 32-row workgroups
    for y, name in ((0, "actor"), (1, "critic")):
        rows = s[y, :g]
        tot = rows[:, 9].mean()
        print(f"{name}: {tot:.0f} cycles per workgroup (wave 0), start spread "
              f"{float(rows[:, 10].max() - rows[:, 10].min()):.0f} cycles")
        for k, ph in enumerate(PHASES):
            print(f"   {rows[:, k].mean():8.0f}  {100 * rows[:, k].mean() / tot:5.1f}%  {ph}")


if __name__ == "__main__":
    main()
