"""GPU: the batched Trainer.evaluation (policy/batched_eval.py) against the sequential one
(trainer.py:266-392 restated in policy/trainer.py), on the same eval configs.

Both paths step the same drop-in envs (host RandomState noise per robot, so the noise streams
are identical); they differ only in the policy call (one batch per step vs batch-1 per robot),
i.e. in GEMM rounding. Episode lengths, successes and times are compared exactly; discounted
returns and energies to 1e-5 relative; trajectories to 1e-6 m. Python's global RNG must end in
the same state (one random.random() per robot action in both)."""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SCHEDULE = {"num_episodes": [3, 3], "num_robots": [3, 5], "num_cores": [0, 0], "num_obstacles": [2, 4],
            "min_start_goal_dis": [30.0, 40.0]}


def _trainer(agent_type):
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.envs.marinenav.env import MarineNavEnv3
    from distributional_rl_decision_and_control_amd.policy.trainer import Trainer
    torch.manual_seed(0)
    agent = Agent(seed=100, agent_type=agent_type)
    train_env = MarineNavEnv3(seed=1)
    eval_env = MarineNavEnv3(seed=253, is_eval_env=True)
    return Trainer(train_env, eval_env, SCHEDULE, agent)


def _run(tr, batched):
    random.seed(77)
    np.random.seed(77)
    tr.evaluation(batched=batched)
    return random.getstate()


@pytest.mark.parametrize("agent_type", ["AC-IQN", "Rainbow"])
def test_batched_evaluation_matches_sequential(agent_type):
    tr = _trainer(agent_type)
    st_seq = _run(tr, False)
    st_bat = _run(tr, True)
    assert st_seq == st_bat
    (r0, r1), (s0, s1) = tr.eval_rewards, tr.eval_successes
    (t0, t1), (e0, e1) = tr.eval_times, tr.eval_energies
    (j0, j1) = tr.eval_trajectories
    (a0, a1) = tr.eval_actions
    assert len(r0) == len(r1) == sum(SCHEDULE["num_episodes"])
    assert s0 == s1
    assert t0 == t1
    np.testing.assert_allclose(r1, r0, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(e1, e0, rtol=1e-5, atol=1e-6)
    for ep0, ep1 in zip(j0, j1):
        for rob0, rob1 in zip(ep0, ep1):
            assert len(rob0) == len(rob1)
            if rob0:
                np.testing.assert_allclose(np.array(rob1, dtype=float), np.array(rob0, dtype=float), atol=1e-6)
    for ep0, ep1 in zip(a0, a1):
        for rob0, rob1 in zip(ep0, ep1):
            assert len(rob0) == len(rob1)
            if rob0:
                np.testing.assert_allclose(np.array(rob1, dtype=float), np.array(rob0, dtype=float), rtol=1e-5,
                                           atol=1e-6)


def test_batched_evaluation_iqn_runs():
    """IQN draws fresh quantile fractions per call (agent.py:240): the batched path is checked for
    completing every config with well-formed metrics and discrete actions."""
    tr = _trainer("IQN")
    tr.evaluation(batched=True)
    n = sum(SCHEDULE["num_episodes"])
    assert len(tr.eval_rewards[0]) == n and len(tr.eval_successes[0]) == n
    for ep in tr.eval_actions[0]:
        for rob in ep:
            assert all(0 <= int(a) < 25 for a in rob)
