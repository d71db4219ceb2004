#!/usr/bin/env python3
"""Wall time of Trainer.evaluation over the reference config's eval schedule (60 episodes,
config/ac_iqn.json), sequential (trainer.py:266-392 one robot at a time) vs batched
(policy/batched_eval.py). Untrained AC-IQN policy, so episodes end early on collisions; the
reported per-step numbers normalise for that.

    python tools/bench_eval.py [--agent AC-IQN] [--skip-sequential]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SCHEDULE = {"num_episodes": [10, 10, 10, 10, 10, 10], "num_robots": [3, 4, 5, 5, 5, 5], "num_cores": [0] * 6,
            "num_obstacles": [0, 0, 0, 2, 3, 4], "min_start_goal_dis": [30.0, 35.0, 40.0, 40.0, 40.0, 40.0]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agent", default="AC-IQN")
    ap.add_argument("--skip-sequential", action="store_true")
    a = ap.parse_args()
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.envs.marinenav.env import MarineNavEnv3
    from distributional_rl_decision_and_control_amd.policy.trainer import Trainer
    torch.manual_seed(0)
    tr = Trainer(MarineNavEnv3(seed=1), MarineNavEnv3(seed=253, is_eval_env=True), SCHEDULE,
                 Agent(seed=100, agent_type=a.agent))
    out = {"episodes": len(tr.eval_config), "agent": a.agent}
    for mode in ([True] if a.skip_sequential else [False, True]):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.evaluation(batched=mode)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        steps = sum(len(r[0]) for r in tr.eval_trajectories[-1])   # robot 0's recorded steps per episode
        key = "batched" if mode else "sequential"
        out[key + "_s"] = el
        out[key + "_env_steps"] = steps
        out[key + "_success_rate"] = float(sum(tr.eval_successes[-1]) / len(tr.eval_successes[-1]))
    if "sequential_s" in out:
        out["speedup"] = out["sequential_s"] / out["batched_s"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
