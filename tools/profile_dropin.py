#!/usr/bin/env python3
"""Host profile (cProfile) of the drop-in path bench.py's dropin_single_env line times: Trainer.learn on one
MarineNavEnv3 with the AC-IQN Agent at the reference's learner shape. Prints the top functions by cumulative and
by own time.

    python tools/profile_dropin.py [--steps 400]
"""
import argparse
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    import contextlib
    import io
    import torch
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.envs.marinenav.env import MarineNavEnv3
    from distributional_rl_decision_and_control_amd.policy.trainer import Trainer
    sched = {"timesteps": [0], "num_robots": [5], "num_cores": [0], "num_obstacles": [4], "min_start_goal_dis": [40.0]}
    env = MarineNavEnv3(seed=0, schedule=sched)
    eval_env = MarineNavEnv3(seed=253, is_eval_env=True)
    agent = Agent(device="cuda", seed=100, agent_type="AC-IQN")
    ev = {"num_episodes": [1], "num_robots": [5], "num_cores": [0], "num_obstacles": [4], "min_start_goal_dis": [40.0]}
    tr = Trainer(train_env=env, eval_env=eval_env, eval_schedule=ev, rl_agent=agent, learning_starts=100)
    tr.evaluation = lambda *x, **k: None
    tr.save_evaluation = lambda *x, **k: None
    agent.save_latest_model = lambda *x, **k: None
    with contextlib.redirect_stdout(io.StringIO()):
        tr.learn(300, 10 ** 12, "/tmp", verbose=False)
        s0 = tr.current_timestep
        pr = cProfile.Profile()
        pr.enable()
        tr.learn(s0 + a.steps, 10 ** 12, "/tmp", verbose=False)
        torch.cuda.synchronize()
        pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(35)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
