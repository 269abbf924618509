"""MI355X-native PPO rollout-and-update engine (gfx950 HIP kernels behind a C-ABI).

Drop-in classes for the reference's hot path (aminrezaee/mujoco_reinforcement_learning):
  PPOEngine              <- entities/algorithms/ppo.py  PPO
  PPOEngineAgent         <- entities/agents/ppo_agent.py PPOAgent
  SyntheticVecEnvHelper  <- environments/helper.py EnvironmentHelper (synthetic dynamics)
  RolloutBuffer          <- the TensorDict rollout memory (ppo.py:30-60)
  Run & configs          <- entities/features.py
"""
from .features import (AgentConfig, DynamicConfig, EngineConfig, EnvironmentConfig, NetworkConfig,
                       PPOConfig, RewardConfig, Run, SACConfig, TrainingConfig)

__all__ = ["AgentConfig", "DynamicConfig", "EngineConfig", "EnvironmentConfig", "NetworkConfig",
           "PPOConfig", "RewardConfig", "Run", "SACConfig", "TrainingConfig", "PPOEngine",
           "PPOEngineAgent", "SyntheticVecEnvHelper", "RolloutBuffer", "make_run"]


def __getattr__(name):
    # GPU-facing classes import the native library lazily (config-only users need no GPU)
    if name == "PPOEngine":
        from .algorithm import PPOEngine
        return PPOEngine
    if name == "PPOEngineAgent":
        from .agent import PPOEngineAgent
        return PPOEngineAgent
    if name == "SyntheticVecEnvHelper":
        from .environments import SyntheticVecEnvHelper
        return SyntheticVecEnvHelper
    if name == "RolloutBuffer":
        from .buffer import RolloutBuffer
        return RolloutBuffer
    if name == "make_run":
        from .runconfig import make_run
        return make_run
    raise AttributeError(name)
