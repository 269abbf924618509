"""Run configuration -- the drop-in for ``entities.features`` (reference features.py:12-165).

Field names and their *positional order* are kept: the reference builds these dataclasses
positionally in main.py:40-108 and restores them positionally from configurations.json
(features.py:145-165), so both keep working against this module.  ``Run`` is the same
process-wide singleton (``Run.instance()``, type_utils.py:1-7).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field
from typing import List, Optional

import torch


class Singleton(type):
    """One instance per class (utils/type_utils.py:1-7)."""
    _instances: dict = {}

    def __call__(cls, *args, **kwargs):
        if cls not in cls._instances:
            cls._instances[cls] = super().__call__(*args, **kwargs)
        return cls._instances[cls]


@dataclass
class RewardConfig:
    pass


@dataclass
class TrainingConfig:
    iteration_count: int
    learning_rate: float
    weight_decay: float          # declared, never read by the reference path
    batch_size: float            # minibatch rows (ppo.py:95-98)
    epochs_per_iteration: int
    minimum_learning_rate: float
    agents_dir: str = "./outputs/agents"
    save_per_iteration: int = 10


@dataclass
class EnvironmentConfig:
    maximum_timesteps: int       # T: rollout horizon per iteration
    num_envs: int                # N
    window_length: int           # W


@dataclass
class AgentConfig:
    sub_action_count: int


@dataclass
class NetworkConfig:
    input_shape: int             # O
    output_shape: int            # A
    output_max_value: float
    activation_class: type
    num_linear_layers: int
    linear_hidden_shapes: List[int]
    num_feature_extractor_layers: int
    feature_extractor_latent_size: int
    use_bias: bool
    use_batch_norm: bool
    feature_extractor: str
    last_layer_std: float


@dataclass
class DynamicConfig:
    current_episode: int
    current_episode_timestep: int
    current_timestep: int
    best_reward: float

    def next_episode(self):
        self.current_episode = int(self.current_episode + 1)

    def next_timestep(self):
        self.current_episode_timestep = int(self.current_episode_timestep + 1)
        self.current_timestep = int(self.current_timestep + 1)

    def reset_timestep(self):
        self.current_episode_timestep = 0

    def set_episode(self, episode: int):
        self.current_episode = episode


@dataclass
class PPOConfig:
    max_grad_norm: float
    clip_epsilon: float
    gamma: float
    lmbda: float
    entropy_eps: float
    advantage_scaler: float
    normalize_advantage: bool
    critic_coeffiecient: float   # (sic) reference spelling, unused by ppo.py


@dataclass
class SACConfig:
    max_grad_norm: float
    gamma: float
    alpha: float
    tau: float
    memory_capacity: int
    target_update_interval: int
    automatic_entropy_tuning: bool


ENGINE_CONFIG_FILE = "engine_configuration.json"


@dataclass
class EngineConfig:
    """Engine-only knobs (not in the reference; defaults reproduce the reference behaviour).

    rng: "torch" draws sampling noise and minibatch permutations from the torch global CPU
         generator in the reference order (bit-for-bit the same draws as ppo.py); "philox" uses
         counter-based Philox normals and a keyed Feistel permutation on the GPU (no host RNG).
    critic_hidden_shapes: hidden widths of the MLP critic; None = the reference critic's
         hard-coded [128, 128] (models/critic.py:10-15), so a drop-in run builds the same critic
         and its networks.pth / optimizer_critic.pth load into the reference's modules.  The
         BASELINE configs ("actor+critic 2x256") set it explicitly (runconfig.make_run).
    seed: key of the philox streams.
    dp_mode: "local" (weak scaling: per-rank shuffles, loss / (B*world)) or "exact" (global
         reference permutation sharded across ranks, loss / B) -- distributed.py.
    rollout_graph: with rng="philox" and a device-resident VecEnv helper (``graph_safe``),
         capture the T-step rollout once as a hipGraph and replay it each iteration (no host
         launch overhead per step; the Philox offset base is a device counter).
    train_graph: with rng="philox" on a single rank, capture the E x M optimizer steps of an
         iteration once as a hipGraph (minibatch rows of all epochs drawn up front, Adam step
         sizes read from a device schedule) and replay it each iteration.
    precision: "f32" (every GEMM in f32, parity with the reference) or "bf16" (fc-layer GEMM
         operands rounded to bf16 with f32 accumulation; params, optimizer state, activations,
         heads, losses and GAE stay f32) -- BASELINE.json configs[1].
    """
    rng: str = "torch"
    critic_hidden_shapes: Optional[List[int]] = None
    seed: int = 0
    dp_mode: str = "local"
    rollout_graph: bool = True
    train_graph: bool = True
    precision: str = "f32"


REFERENCE_CRITIC_HIDDEN = (128, 128)  # models/critic.py:14


@dataclass
class Run(metaclass=Singleton):
    rewards_config: RewardConfig
    training_config: TrainingConfig
    ppo_config: PPOConfig
    sac_config: SACConfig
    environment_config: EnvironmentConfig
    agent_config: AgentConfig
    network_config: NetworkConfig
    dynamic_config: DynamicConfig
    processors: int
    device: str
    experiment_path: str
    verbose: bool
    central_critic: bool
    central_actor: bool
    normalize_rewards: bool
    normalize_actions: bool
    normalize_observations: bool
    sequence_wise_normalization: bool
    dtype: torch.dtype
    render_size: List[int]
    engine_config: EngineConfig = field(default_factory=EngineConfig)

    def get_name(self):
        return "_".join(f"{k}" for k in sorted(asdict(self)))

    @staticmethod
    def instance() -> Optional["Run"]:
        inst = Singleton._instances.get(Run)
        return inst

    @staticmethod
    def reset_instance() -> None:
        Singleton._instances.pop(Run, None)

    def save(self):
        """features.py:134-143: configurations.json in the reference's exact schema (its
        get_configurations restores Run positionally, so an extra key would break a reference
        resume); the engine-only knobs go to engine_configuration.json beside it."""
        cfg = {"run": asdict(self)}
        engine = cfg["run"].pop("engine_config")
        if engine.get("critic_hidden_shapes") is None:  # persist the critic widths explicitly
            engine["critic_hidden_shapes"] = list(REFERENCE_CRITIC_HIDDEN)
        cfg["run"]["dtype"] = str(cfg["run"]["dtype"]).split(".")[-1]
        cfg["run"]["network_config"]["activation_class"] = (
            self.network_config.activation_class.__name__)
        os.makedirs(self.experiment_path, exist_ok=True)
        with open(f"{self.experiment_path}/configurations.json", "w") as fh:
            fh.write(json.dumps(cfg, indent=4))
        with open(f"{self.experiment_path}/{ENGINE_CONFIG_FILE}", "w") as fh:
            fh.write(json.dumps(engine, indent=4))

    @staticmethod
    def get_configurations(experiment_path: str) -> "Run":
        with open(f"{experiment_path}/configurations.json") as fh:
            cfg = json.load(fh)["run"]
        cfg["dtype"] = getattr(torch, cfg["dtype"])
        cfg["network_config"]["activation_class"] = getattr(
            torch.nn, cfg["network_config"]["activation_class"])
        parts = [
            RewardConfig(*cfg.pop("rewards_config").values()),
            TrainingConfig(*cfg.pop("training_config").values()),
            PPOConfig(*cfg.pop("ppo_config").values()),
            SACConfig(*cfg.pop("sac_config").values()),
            EnvironmentConfig(*cfg.pop("environment_config").values()),
            AgentConfig(*cfg.pop("agent_config").values()),
            NetworkConfig(*cfg.pop("network_config").values()),
            DynamicConfig(*cfg.pop("dynamic_config").values()),
        ]
        engine_kw = cfg.pop("engine_config", None)
        if engine_kw is not None and engine_kw.get("critic_hidden_shapes") is None:
            # a run directory of the earlier format embedded engine_config, where a null critic
            # width meant "the actor's widths": keep building the critic it saved
            nc = parts[6]
            engine_kw["critic_hidden_shapes"] = [
                int(h) for h in list(nc.linear_hidden_shapes)[:nc.num_linear_layers]]
        side = f"{experiment_path}/{ENGINE_CONFIG_FILE}"
        if engine_kw is None and os.path.exists(side):
            with open(side) as fh:
                engine_kw = json.load(fh)
        engine = EngineConfig(**(engine_kw or {}))  # a reference run dir: engine defaults
        Run.reset_instance()
        return Run(*parts, *cfg.values(), engine_config=engine)
