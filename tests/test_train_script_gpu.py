"""Plumbing: the reference CLI flow (config JSON -> trials -> Trainer.learn with evaluation
and checkpointing) through the GPU-backed surfaces, at a reduced size (SURVEY.md 8d, config 1:
same artefact files, exit code 0)."""
import glob
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = {
    "seed": [0], "total_timesteps": 2020, "eval_freq": 60000, "save_dir": None,
    "training_schedule": {"timesteps": [0], "num_robots": [3], "num_cores": [0], "num_obstacles": [2],
                          "min_start_goal_dis": [30.0]},
    "eval_schedule": {"num_episodes": [1], "num_robots": [3], "num_cores": [0], "num_obstacles": [2],
                      "min_start_goal_dis": [30.0]},
    "imitation_learning": False, "agent_type": None,
}


@pytest.mark.parametrize("agent_type,files", [
    ("AC-IQN", ["actor_network_params.pth", "actor_constructor_params.json", "critic_network_params.pth",
                "critic_constructor_params.json"]),
    ("IQN", ["network_params.pth", "constructor_params.json"]),
    ("DQN", ["network_params.pth", "constructor_params.json"]),   # BASELINE config 1
])
def test_train_rl_agents_cli(tmp_path, agent_type, files):
    from distributional_rl_decision_and_control_amd.scripts import train_RL_agents as cli
    cfg = dict(CFG, save_dir=str(tmp_path), agent_type=agent_type)
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    cli.main(["-C", str(p), "-D", "cpu"])
    runs = glob.glob(str(tmp_path / "training_*" / "seed_0"))
    assert len(runs) == 1
    d = runs[0]
    for f in ["trial_config.json", "eval_configs.json", "evaluations.npz"] + files:
        assert os.path.exists(os.path.join(d, f)), f
    ev = np.load(os.path.join(d, "evaluations.npz"), allow_pickle=True)  # our own file
    assert list(ev["timesteps"]) == [2000]
    # checkpoint round trip through the reference's loader convention
    from distributional_rl_decision_and_control_amd.agent import Agent
    ag = Agent(agent_type=agent_type)
    ag.load_model(d)
    assert next(iter(ag.policy_local.parameters() if agent_type != "AC-IQN" else ag.policy_local.actor.parameters())).is_cuda


@pytest.mark.parametrize("agent_type", ["AC-IQN", "IQN"])
def test_cli_schedule_key_routes_to_batched_loop(tmp_path, agent_type):
    """The reference's run_trial passes training_schedule unchanged into MarineNavEnv3
    (train_RL_agents.py:85); with the extra "vectorized" key (ignored by the reference) the drop-in
    Trainer.learn drives VecTrainer: same artefacts, evaluation at the first learning iteration and at
    every eval_freq crossing, and the saved networks are the batched loop's trained ones."""
    from distributional_rl_decision_and_control_amd.scripts import train_RL_agents as cli
    from distributional_rl_decision_and_control_amd.policy import trainer as trainer_mod
    sched = dict(CFG["training_schedule"], vectorized={"n_envs": 128, "batch_size": 512, "num_tau": 32})
    cfg = dict(CFG, save_dir=str(tmp_path), agent_type=agent_type, total_timesteps=128 * 20, eval_freq=128 * 10,
               training_schedule=sched)
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    seen = {}
    orig = trainer_mod.Trainer.learn_vectorized

    def spy(self, *a, **k):
        tr = orig(self, *a, **k)
        seen["tr"] = tr
        return tr
    trainer_mod.Trainer.learn_vectorized = spy
    try:
        cli.main(["-C", str(p), "-D", "cpu"])
    finally:
        trainer_mod.Trainer.learn_vectorized = orig
    tr = seen["tr"]
    assert tr.E == 128 and tr.B == 512 and tr.learn_steps > 10
    assert (tr.fused2 if agent_type == "AC-IQN" else tr.fused_iqn) is not None   # the fused learner ran
    d = glob.glob(str(tmp_path / "training_*" / "seed_0"))[0]
    for f in ["trial_config.json", "eval_configs.json", "evaluations.npz"]:
        assert os.path.exists(os.path.join(d, f)), f
    ev = np.load(os.path.join(d, "evaluations.npz"), allow_pickle=True)  # our own file
    ts = list(ev["timesteps"])
    assert len(ts) == 3 and ts == sorted(ts) and ts[-1] == 128 * 20   # first learning iteration, 1280, 2560
    from distributional_rl_decision_and_control_amd.agent import Agent
    ag = Agent(agent_type=agent_type)
    ag.load_model(d)
    src = tr.local.actor if agent_type == "AC-IQN" else tr.local
    dst = ag.policy_local.actor if agent_type == "AC-IQN" else ag.policy_local
    for (n1, a), (n2, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert n1 == n2 and torch.equal(a.cpu(), b.cpu()), n1
    fresh = Agent(agent_type=agent_type, seed=100)
    fp = fresh.policy_local.actor if agent_type == "AC-IQN" else fresh.policy_local
    assert any(not torch.equal(a.cpu(), b.cpu()) for a, b in zip(fp.parameters(), dst.parameters()))
