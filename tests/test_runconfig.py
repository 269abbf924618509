"""CPU: Run.save / Run.get_configurations round trips of the engine's run directory
(features.py:134-165 schema; the engine-only knobs live in engine_configuration.json)."""
import dataclasses
import json

from mujoco_reinforcement_learning_amd.features import ENGINE_CONFIG_FILE, Run
from mujoco_reinforcement_learning_amd.runconfig import make_run


def test_save_persists_explicit_critic_widths(tmp_path):
    run = make_run(num_envs=8, horizon=4, hidden=(64, 64), experiment_path=str(tmp_path))
    run.engine_config.critic_hidden_shapes = None  # "the reference critic" (models/critic.py:14)
    run.save()
    with open(tmp_path / ENGINE_CONFIG_FILE) as fh:
        assert json.load(fh)["critic_hidden_shapes"] == [128, 128]
    back = Run.get_configurations(str(tmp_path))
    assert back.engine_config.critic_hidden_shapes == [128, 128]
    assert back.network_config.linear_hidden_shapes == [64, 64]


def test_old_format_embedded_null_critic_means_actor_widths(tmp_path):
    """A run directory written by the earlier format embedded engine_config in
    configurations.json, and critic_hidden_shapes null meant the actor's widths: restoring it
    must rebuild that critic (else networks.pth no longer loads)."""
    run = make_run(num_envs=8, horizon=4, hidden=(64, 32), experiment_path=str(tmp_path))
    cfg = {"run": dataclasses.asdict(run)}
    cfg["run"]["dtype"] = "float32"
    cfg["run"]["network_config"]["activation_class"] = "ReLU"
    cfg["run"]["engine_config"]["critic_hidden_shapes"] = None
    with open(tmp_path / "configurations.json", "w") as fh:
        json.dump(cfg, fh)
    back = Run.get_configurations(str(tmp_path))
    assert back.engine_config.critic_hidden_shapes == [64, 32]
    Run.reset_instance()
