"""GPU: the batched Trainer.evaluation (policy/batched_eval.py: every eval config in one asvrl_env_step
batch, one batched greedy policy call per step) against the reference's own Trainer.evaluation
(trainer.py:266-392), captured by tools/capture_oracle.py (F9, tests/golden/eval_ref.npz): the
reference's seeded initial AC-IQN and Rainbow agents, greedy, batch-1 CPU policy per robot, on the
eval configs of a two-entry schedule (3 robots / 2 buoys, and 5 robots / 4 buoys / 2 vortex cores).
The drop-in sequential evaluation (batched=False: the reference's loop over configs and robots,
env steps through the same kernel) is held to the same bars.

Same configs and weights (loaded from the fixture), same seeds. Per config: episode length, success
and time exact; discounted return and energy within 1e-5 relative (the north star's return bar). The
policies differ only in f32 GEMM rounding (batched GPU vs batch-1 CPU), which the closed loop carries
forward over up to 1000 steps: per-robot trajectory entries (pose, velocities, thrusts) within 1e-3
absolute and actions within 1e-3. Observed: AC-IQN actions 1.8e-6, trajectory entries 7.4e-4, returns
1.4e-7 relative; Rainbow (discrete, identical actions) trajectories 5e-12, returns 7e-16.
"""
import json
import random

import numpy as np
import pytest
import torch

from oracle import env_oracle as eo

pytestmark = pytest.mark.gpu

SCHEDULE = {"num_episodes": [2, 2], "num_robots": [3, 5], "num_cores": [0, 2], "num_obstacles": [2, 4],
            "min_start_goal_dis": [30.0, 40.0]}   # tools/capture_oracle.py EVAL_SCHEDULE


@pytest.mark.parametrize("batched", [True, False])
@pytest.mark.parametrize("kind", ["AC-IQN", "Rainbow"])
def test_evaluation_matches_reference(kind, batched):
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.envs.marinenav.env import MarineNavEnv3
    from distributional_rl_decision_and_control_amd.policy.trainer import Trainer
    z = np.load(eo.GOLDEN + "/eval_ref.npz")
    p = kind + "/"
    torch.manual_seed(0)
    agent = Agent(seed=100, agent_type=kind)
    net = agent.policy_local.actor if kind == "AC-IQN" else agent.policy_local
    sd = {k[len(p + "net/"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(p + "net/")}
    net.load_state_dict(sd)
    tr = Trainer(MarineNavEnv3(seed=1), MarineNavEnv3(seed=253, is_eval_env=True), SCHEDULE, agent)
    configs = json.loads(str(z[p + "configs"]))
    assert len(configs) == len(tr.eval_config)
    tr.eval_config = configs
    random.seed(77)
    np.random.seed(77)
    tr.evaluation(batched=batched)
    rewards, successes = np.array(tr.eval_rewards[0]), np.array(tr.eval_successes[0])
    times, energies = np.array(tr.eval_times[0]), np.array(tr.eval_energies[0])
    np.testing.assert_array_equal(successes, z[p + "successes"])
    np.testing.assert_array_equal(times, z[p + "times"])
    np.testing.assert_allclose(rewards, z[p + "rewards"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(energies, z[p + "energies"], rtol=1e-5, atol=1e-9)
    dt_max = da_max = 0.0
    for e, ep in enumerate(tr.eval_trajectories[0]):
        for i, traj in enumerate(ep):
            ref_t, ref_a = z[f"{p}traj/{e}/{i}"], z[f"{p}act/{e}/{i}"]
            got_t = np.array(traj, dtype=np.float64)
            got_a = np.array(tr.eval_actions[0][e][i], dtype=np.float64)
            assert got_t.shape == ref_t.shape and got_a.shape == ref_a.shape, (e, i)
            if got_t.size:
                dt_max = max(dt_max, float(np.abs(got_t - ref_t).max()))
                np.testing.assert_allclose(got_t, ref_t, rtol=0, atol=1e-3, err_msg=f"trajectory {e}/{i}")
            if got_a.size:
                da_max = max(da_max, float(np.abs(got_a - ref_a).max()))
                np.testing.assert_allclose(got_a, ref_a, rtol=0, atol=1e-3, err_msg=f"actions {e}/{i}")
    print(f"{kind} batched={batched}: max |trajectory diff| {dt_max:.2e}, max |action diff| {da_max:.2e}, "
          f"max return rel diff {np.abs(rewards / z[p + 'rewards'] - 1).max():.2e}")
