"""Build a ``Run`` for the PPO hot path (the configs of BASELINE.json / main.py:40-108)."""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .features import (AgentConfig, DynamicConfig, EngineConfig, EnvironmentConfig, NetworkConfig,
                       PPOConfig, RewardConfig, Run, SACConfig, TrainingConfig)

_ACT = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh, "elu": torch.nn.ELU}


def make_run(num_envs: int = 4096, horizon: int = 128, obs_dim: int = 17, act_dim: int = 6,
             window: int = 1, hidden: Sequence[int] = (256, 256),
             critic_hidden: Optional[Sequence[int]] = None, activation: str = "relu",
             batch_size: int = 65536, epochs: int = 10, learning_rate: float = 1e-4,
             gamma: float = 0.99, lmbda: float = 0.98, clip_epsilon: float = 0.1,
             entropy_eps: float = 1e-4, normalize_advantage: bool = False,
             normalize_rewards: bool = False, normalize_observations: bool = True,
             advantage_scaler: float = 1.0, use_bias: bool = True, output_max_value: float = 1.0,
             rng: str = "torch", seed: int = 0, dp_mode: str = "local",
             rollout_graph: bool = True, train_graph: bool = True, precision: str = "f32",
             experiment_path: str = "/tmp/ppo_engine_run",
             feature_extractor: str = "MLP", latent: int = 256, extractor_layers: int = 1,
             replace: bool = True) -> Run:
    """Defaults: the headline HalfCheetah config (BASELINE.json configs[1]) with main.py's PPO
    hyper-parameters (lr 1e-4, gamma 0.99, lambda 0.98, clip 0.1, entropy 1e-4, E=10).

    critic_hidden: None -> the actor's widths (the BASELINE configs name one MLP shape for actor
    and critic); pass "reference" for the reference critic's hard-coded [128, 128]
    (models/critic.py:14, main.py's network).
    feature_extractor="LSTM" selects the reference PPOAgent's BiLSTM actor / critic
    (latent = feature_extractor_latent_size, extractor_layers = num_feature_extractor_layers;
    main.py:63-75 uses 256 and 1); their MLPs use ``hidden``."""
    if critic_hidden is None:
        critic_hidden = hidden
    elif critic_hidden == "reference":
        critic_hidden = (128, 128)
    if replace:
        Run.reset_instance()
    return Run(RewardConfig(),
               TrainingConfig(iteration_count=1, learning_rate=learning_rate, weight_decay=1e-4,
                              batch_size=batch_size, epochs_per_iteration=epochs,
                              minimum_learning_rate=learning_rate),
               PPOConfig(max_grad_norm=1.0, clip_epsilon=clip_epsilon, gamma=gamma, lmbda=lmbda,
                         entropy_eps=entropy_eps, advantage_scaler=advantage_scaler,
                         normalize_advantage=normalize_advantage, critic_coeffiecient=1.0),
               SACConfig(1.0, 0.99, 0.05, 0.005, 999, 1, False),
               EnvironmentConfig(maximum_timesteps=horizon, num_envs=num_envs,
                                 window_length=window),
               AgentConfig(sub_action_count=1),
               NetworkConfig(input_shape=obs_dim, output_shape=act_dim,
                             output_max_value=output_max_value, activation_class=_ACT[activation],
                             num_linear_layers=len(hidden), linear_hidden_shapes=list(hidden),
                             num_feature_extractor_layers=extractor_layers,
                             feature_extractor_latent_size=latent,
                             use_bias=use_bias, use_batch_norm=False,
                             feature_extractor=feature_extractor,
                             last_layer_std=0.01),
               DynamicConfig(0, 0, 0, 0), processors=1, device="cuda",
               experiment_path=experiment_path, verbose=False, central_critic=True,
               central_actor=True, normalize_rewards=normalize_rewards, normalize_actions=False,
               normalize_observations=normalize_observations, sequence_wise_normalization=False,
               dtype=torch.float32, render_size=[200, 200],
               engine_config=EngineConfig(rng=rng,
                                          critic_hidden_shapes=[int(h) for h in critic_hidden],
                                          seed=seed,
                                          dp_mode=dp_mode, rollout_graph=rollout_graph,
                                          train_graph=train_graph,
                                          precision=precision))
