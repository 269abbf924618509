"""Per-phase cycle breakdown of the fused bf16 update kernel (diagnostic stamped build).

Runs headline-shape minibatches (B=65536, 2x256 ReLU) through ppo_minibatch_grad with
ppo_ctx_phase_stamps enabled and prints, for actor and critic workgroups, the mean s_memtime
cycles per phase segment summed over a workgroup's chunks (wave 0's view: a segment that ends at
a barrier includes waiting for the slowest wave).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

SEGMENTS = ["0 X stage + W0 frags", "1 L0 fwd (+ W1 ring prime)", "2 L1 fwd MFMA pass",
            "3 bias/act -> A2 image (+ row scalars to LDS)", "4 head z on MFMA + loss (waves 0-3)",
            "5 d2 = dz.Wh + head dW (MFMA) + D2 image", "6 dW1 wgrad (MFMA, tr reads)",
            "7 dgrad MFMA pass", "8 dgrad epilogue (act', D1 image, bias)", "9 dW0 wgrad",
            "10 prologue (LDS images, constants)", "11 epilogue: slab stores drained"]


def main():
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
    segments = SEGMENTS
    res = {}
    for rep in range(3):
        E.feistel_rows(1, rep, 0, b, n, t, rows)
        eng.phase_stamps(True)
        eng.minibatch_grad(states, actions, logp, adv, vt, rows, b, agent.flat_grad, loss,
                           0.9, 1.1, 1e-4, 1 / b, 1 / (b * 6))
        st = eng.phase_stamps(False).double()
        cyc, real = st[..., :12], st[..., 12]
        res = {"actor": cyc[0].mean(0).tolist(), "critic": cyc[1].mean(0).tolist(),
               "actor_total_max": float(cyc[0].sum(1).max()),
               "critic_total_max": float(cyc[1].sum(1).max()),
               # s_memtime / s_memrealtime x 100 MHz: the shader clock during the launch
               "clock_mhz": float((cyc.sum(-1) / real.clamp_min(1)).median() * 100.0),
               "body_us_max": float(real.max()) / 100.0}
    print(f"clock {res['clock_mhz']:.0f} MHz, slowest workgroup body {res['body_us_max']:.1f} us")
    for k in ("actor", "critic"):
        tot = sum(res[k])
        print(f"{k}: total {tot:.0f} cycles/WG (max {res[k + '_total_max']:.0f})")
        for name, v in zip(segments, res[k]):
            print(f"   {v:10.0f}  {100 * v / max(tot, 1):5.1f}%  {name}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "fused_phases.json"), "w") as f:
        json.dump({"segments": segments, **res}, f, indent=1)


if __name__ == "__main__":
    main()
