"""Generate tests/golden/reference_lstm.npz from the REFERENCE's own LSTM actor / critic.

Run here (the container that has /root/reference), never on the GPU box:

    python tests/golden/gen_golden_lstm.py

It imports ``models.lstm.lstm_actor.LSTMActor`` and ``models.lstm.lstm_critic.LSTMCritic`` from
/root/reference/src (both import with torch only -- SURVEY.md s8(c)), builds them under fixed
``torch.manual_seed`` values in the PPOAgent order (actor, then critic: ppo_agent.py:12-13) and
records, per case:
  meta        [seed, obs, window, act, latent, layers, n_hidden, *hidden]
  activation  the activation name
  x           a fixed (B, W, O) input
  mean / std / value       the reference forward outputs on x; std is row 0 of the reference's
                           (B, B, A) std (lstm_actor.py:48 repeats the per-row (B, A) std B times)
  y_actor / y_critic       the BiLSTM outputs feature_extractor(x)[0]
  actions, old_logp, adv, vt   a PPO minibatch (ppo.py:108-133 inputs)
  loss        [actor_loss, critic_loss] of ppo.py:113-131 with the per-row std
  grad        d(actor_loss + critic_loss)/d(params), actor then critic, parameters() order
              (small cases; the main.py-sized case keeps per-tensor grad_norm / grad_absmax)
  sha256/<name>   digest of every parameter (the init pin); <name> the parameter (small cases)
Only data (inputs, expected outputs, digests) is written: no reference source travels.
"""
import hashlib
import os
import sys

import numpy as np
import torch

REF_SRC = "/root/reference/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_lstm.npz")
FULL_PARAMS_LIMIT = 200_000

CASES = [
    # name, seed, obs, window, act, latent, layers, hidden, activation, batch
    ("lstm_relu_small", 21, 17, 3, 6, 8, 1, [16, 16], "ReLU", 24),
    ("lstm_tanh_2layer", 22, 11, 4, 3, 12, 2, [20, 24], "Tanh", 20),
    ("lstm_elu_w1", 23, 27, 1, 8, 16, 1, [32], "ELU", 16),
    # the reference's own network (main.py:63-75): O=348, W=5, latent 256, 1 layer,
    # [256, 256, 128, 128], A=17, ReLU
    ("lstm_main_py", 24, 348, 5, 17, 256, 1, [256, 256, 128, 128], "ReLU", 8),
]


def _make_run(obs, window, act, latent, layers, hidden, activation):
    from entities import features as F
    F.Run._instances.clear()
    net = F.NetworkConfig(input_shape=obs, output_shape=act, output_max_value=1.0,
                          activation_class=getattr(torch.nn, activation),
                          num_linear_layers=len(hidden), linear_hidden_shapes=list(hidden),
                          num_feature_extractor_layers=layers,
                          feature_extractor_latent_size=latent, use_bias=True,
                          use_batch_norm=False, feature_extractor="LSTM", last_layer_std=0.01)
    return F.Run(F.RewardConfig(), F.TrainingConfig(1, 1e-4, 1e-4, 64, 10, 1e-4),
                 F.PPOConfig(1.0, 0.1, 0.99, 0.98, 1e-4, 1.0, False, 1.0),
                 F.SACConfig(1.0, 0.99, 0.05, 0.005, 999, 1, False),
                 F.EnvironmentConfig(16, 8, window), F.AgentConfig(1), net,
                 F.DynamicConfig(0, 0, 0, 0), processors=1, device="cpu", experiment_path="/tmp",
                 verbose=False, central_critic=True, central_actor=True, normalize_rewards=False,
                 normalize_actions=False, normalize_observations=True,
                 sequence_wise_normalization=False, dtype=torch.float32, render_size=[8, 8])


def main():
    sys.path.insert(0, REF_SRC)
    from models.lstm.lstm_actor import LSTMActor
    from models.lstm.lstm_critic import LSTMCritic

    out = {}
    for name, seed, obs, window, act, latent, layers, hidden, activation, batch in CASES:
        _make_run(obs, window, act, latent, layers, hidden, activation)
        torch.manual_seed(seed)
        actor = LSTMActor()
        critic = LSTMCritic()
        gen = torch.Generator().manual_seed(2000 + seed)
        x = torch.randn(batch, window, obs, generator=gen)
        actions = torch.randn(batch, act, generator=gen) * 0.3
        adv = torch.randn(batch, 1, generator=gen)
        vt = torch.randn(batch, 1, generator=gen) * 2.0
        with torch.no_grad():
            mean0, std0 = actor(x)
            lp0 = torch.distributions.Normal(mean0, std0[0]).log_prob(actions).sum(dim=1)
        # old log-probs around the current ones: ratios on both sides of the clip range
        old_logp = lp0 + 0.15 * torch.randn(batch, generator=gen)
        mean, std_bug = actor(x)
        std = std_bug[0]  # the per-row (B, A) std the reference repeats B times
        value = critic(x)
        dist = torch.distributions.Normal(mean, std)
        new_logp = dist.log_prob(actions).sum(dim=1)
        critic_loss = torch.nn.functional.huber_loss(value, vt, reduction="mean")
        ratio = (new_logp - old_logp).exp()[:, None]
        s1 = ratio * adv
        s2 = torch.clamp(ratio, 0.9, 1.1) * adv
        actor_loss = -torch.min(s1, s2).mean() - dist.entropy().mean() * 1e-4
        (actor_loss + critic_loss).backward()
        params = list(actor.named_parameters()) + list(critic.named_parameters())
        names = [f"actor.{k}" for k, _ in actor.named_parameters()] + \
                [f"critic.{k}" for k, _ in critic.named_parameters()]
        small = sum(p.numel() for _, p in params) < FULL_PARAMS_LIMIT
        out[f"{name}/meta"] = np.array([seed, obs, window, act, latent, layers, len(hidden),
                                        *hidden], dtype=np.int64)
        out[f"{name}/activation"] = np.array(activation.lower())
        out[f"{name}/names"] = np.array(names)
        for k, v in (("x", x), ("mean", mean), ("std", std), ("value", value),
                     ("actions", actions), ("old_logp", old_logp), ("adv", adv), ("vt", vt)):
            out[f"{name}/{k}"] = v.detach().numpy()
        with torch.no_grad():
            out[f"{name}/y_actor"] = actor.feature_extractor(x)[0].numpy()
            out[f"{name}/y_critic"] = critic.feature_extractor(x)[0].numpy()
        out[f"{name}/loss"] = np.array([float(actor_loss), float(critic_loss)], dtype=np.float64)
        grads = [p.grad.detach().reshape(-1) for _, p in params]
        if small:
            out[f"{name}/grad"] = torch.cat(grads).numpy()
        out[f"{name}/grad_norm"] = np.array([float(g.double().norm()) for g in grads])
        out[f"{name}/grad_absmax"] = np.array([float(g.abs().max()) for g in grads])
        for k, (_, p) in zip(names, params):
            arr = p.detach().contiguous().numpy()
            out[f"{name}/sha256/{k}"] = np.array(hashlib.sha256(arr.tobytes()).hexdigest())
            if small:
                out[f"{name}/param/{k}"] = arr
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, sum(v.nbytes for v in out.values()), "bytes raw")


if __name__ == "__main__":
    main()
