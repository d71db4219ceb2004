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


@pytest.mark.parametrize("agent_type", ["AC-IQN", "IQN", "Rainbow"])
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
    fused = {"AC-IQN": tr.fused2, "IQN": tr.fused_iqn, "Rainbow": tr.fused_rb}[agent_type]
    assert fused is not None   # the fused learner ran
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


def test_cli_vectorized_starts_from_loaded_model(tmp_path):
    """run_trial's load_model (train_RL_agents.py:92-93 -> agent.py:684-698) with the "vectorized" key: the
    batched loop starts from the loaded networks (VecTrainer.load_policies), not its own initialisation,
    and the Trainer's learning_starts / target_update_interval reach it (in transitions / learn steps)."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.policy import trainer as trainer_mod
    from distributional_rl_decision_and_control_amd.scripts import train_RL_agents as cli
    src = Agent(agent_type="AC-IQN", seed=5)
    ck = tmp_path / "ck"
    ck.mkdir()
    src.save_latest_model(str(ck))
    sched = dict(CFG["training_schedule"], vectorized={"n_envs": 128, "batch_size": 512, "num_tau": 32})
    cfg = dict(CFG, save_dir=str(tmp_path), agent_type="AC-IQN", total_timesteps=128 * 2, eval_freq=128 * 10,
               training_schedule=sched, load_model=str(ck))
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    seen = {}
    orig = trainer_mod.Trainer.learn_vectorized

    def spy(self, *a, **k):
        tr = orig(self, *a, **k)
        seen["tr"], seen["trainer"] = tr, self
        return tr
    trainer_mod.Trainer.learn_vectorized = spy
    try:
        cli.main(["-C", str(p), "-D", "cpu"])
    finally:
        trainer_mod.Trainer.learn_vectorized = orig
    tr, trainer = seen["tr"], seen["trainer"]
    assert tr.learn_steps == 0   # two iterations: the replay is still below learning_starts
    assert tr.learning_starts == max(512, trainer.learning_starts)
    assert tr.target_update_interval == trainer.target_update_interval // trainer.UPDATE_EVERY
    for a, b in zip(src.policy_local.actor.parameters(), tr.local.actor.parameters()):
        assert torch.equal(a.cpu(), b.cpu())
    for a, b in zip(src.policy_local.critic.parameters(), tr.local.critic.parameters()):
        assert torch.equal(a.cpu(), b.cpu())
    # the fused act kernel reads the re-packed images: its greedy actions are the loaded actor's
    from distributional_rl_decision_and_control_amd.fused_mlp import actor_forward
    x = tr.env.obs_cur[:256]
    a_kernel = torch.empty(256, 2, device="cuda")
    actor_forward(tr.fused2.actor, x, a_kernel)
    with torch.no_grad():
        a_ref = src.policy_local.actor((x[:, 0:7], x[:, 7:32].reshape(-1, 5, 5), x[:, 32:37]))
    assert (a_kernel - a_ref).abs().max().item() < 2e-2   # the bf16 build's bar (test_fused_mlp_gpu)
