"""Generate tests/golden/reference_mlp.npz from the REFERENCE's own model modules.

Run here (the container that has /root/reference), never on the GPU box:

    python tests/golden/gen_golden.py

It imports ``models.linear.actor.Actor`` and ``models.network_block_creator.create_network`` from
/root/reference/src (both import cleanly with torch only -- SURVEY.md s8(c)), builds them under
fixed ``torch.manual_seed`` values in the PPOAgent order (actor, then critic:
ppo_agent.py:12-14), and records, per case:
  meta        [seed, obs, window, act, n_actor_hidden, n_critic_hidden, *actor, *critic]
  activation  the activation name ("relu" / "tanh" / "elu")
  x           a fixed (32, W, O) input
  mean / std / value   the reference forward outputs on x
  sha256/<state_dict key>   digest of every parameter's bytes (the init pin)
  <state_dict key>          the parameter itself, for the small nets only (< 200 k values)
The critic is the reference ``NetworkBlock`` with ``output_shape=1`` and the window flattened (the
coherent MLP critic of SURVEY.md s0 / s8(b)); its widths are the reference critic's hard-coded
[128, 128] (models/critic.py:14) for main.py's network, the actor's widths for the BASELINE
configs.  Only data (inputs, expected outputs, digests) is written: no reference source travels.
"""
import hashlib
import os
import sys

import numpy as np
import torch

REF_SRC = "/root/reference/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_mlp.npz")
FULL_PARAMS_LIMIT = 200_000

CASES = [
    # name, seed, obs, window, act, actor hidden, critic hidden, activation
    ("relu_2x64", 0, 17, 1, 6, [64, 64], [64, 64], "ReLU"),
    ("tanh_2x64_w2", 1, 17, 2, 6, [64, 64], [64, 64], "Tanh"),
    ("elu_2x32_ant", 2, 27, 1, 8, [32, 32], [32, 32], "ELU"),
    ("relu_2x256", 3, 17, 1, 6, [256, 256], [256, 256], "ReLU"),
    # BASELINE configs[2] Ant-v4 and configs[3] Humanoid-v4 shapes
    ("ant_relu_2x256", 6, 27, 1, 8, [256, 256], [256, 256], "ReLU"),
    ("humanoid_relu_3x512", 4, 376, 1, 17, [512, 512, 512], [512, 512, 512], "ReLU"),
    # the reference's own network (main.py:63-75): O=348, W=5, [256,256,128,128], A=17, ReLU,
    # critic [128, 128] (models/critic.py:14)
    ("main_py_net", 5, 348, 5, 17, [256, 256, 128, 128], [128, 128], "ReLU"),
]


def _make_run(obs, window, act, hidden, activation):
    from entities import features as F
    F.Run._instances.clear()
    net = F.NetworkConfig(input_shape=obs, output_shape=act, output_max_value=1.0,
                          activation_class=getattr(torch.nn, activation),
                          num_linear_layers=len(hidden), linear_hidden_shapes=list(hidden),
                          num_feature_extractor_layers=1, feature_extractor_latent_size=256,
                          use_bias=True, use_batch_norm=False, feature_extractor="MLP",
                          last_layer_std=0.01)
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
    from models.linear.actor import Actor
    from models.network_block_creator import create_network

    out = {}
    for name, seed, obs, window, act, hidden, critic_hidden, activation in CASES:
        run = _make_run(obs, window, act, hidden, activation)
        torch.manual_seed(seed)
        actor = Actor()
        critic_cfg = {"final_activation": None, "activation": run.network_config.activation_class,
                      "hidden_layer_count": len(critic_hidden), "shapes": list(critic_hidden)}
        critic = create_network(critic_cfg, input_shape=obs * window, output_shape=1,
                                normalize_at_the_end=False, use_bias=True)
        gen = torch.Generator().manual_seed(1000 + seed)
        x = torch.randn(32, window, obs, generator=gen)
        with torch.no_grad():
            mean, std = actor(x)
            value = critic(x.reshape(len(x), -1))
        out[f"{name}/x"] = x.numpy()
        out[f"{name}/mean"] = mean.numpy()
        out[f"{name}/std"] = std.numpy()
        out[f"{name}/value"] = value.numpy()
        out[f"{name}/activation"] = np.array(activation.lower())
        sd = {f"actor.{k}": v for k, v in actor.state_dict().items()}
        sd.update({f"critic.network.{k}": v for k, v in critic.state_dict().items()})
        small = sum(v.numel() for v in sd.values()) < FULL_PARAMS_LIMIT
        for k, v in sd.items():
            arr = v.detach().contiguous().numpy()
            out[f"{name}/sha256/{k}"] = np.array(hashlib.sha256(arr.tobytes()).hexdigest())
            if small:
                out[f"{name}/{k}"] = arr
        out[f"{name}/meta"] = np.array([seed, obs, window, act, len(hidden), len(critic_hidden),
                                        *hidden, *critic_hidden], dtype=np.int64)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, sum(v.nbytes for v in out.values()), "bytes raw")


if __name__ == "__main__":
    main()
