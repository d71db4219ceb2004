"""train_RL_agents -- the reference CLI (rfarl/rfarl/scripts/train_RL_agents.py:1-141) on
the GPU-backed env/agent/trainer.

    python -m distributional_rl_decision_and_control_amd.scripts.train_RL_agents -C config/ac_iqn.json [-P n] [-D dev]

Same flags, the same config JSON schema (list-valued keys expand to a cartesian product of
trials), the same per-trial directory layout and artefacts, and run_trial is the reference's
(train_RL_agents.py:74-109). The batched GPU loop is reached through an optional key the reference
ignores: "training_schedule": {..., "vectorized": {"n_envs": E, "batch_size": B, ...}} -- the
schedule goes into MarineNavEnv3 unchanged and the drop-in Trainer.learn drives VecTrainer when the
key is present (policy/trainer.py). A top-level "vectorized" entry is moved into the schedule.
Trials run in spawned worker processes (HIP-safe) and worker errors are re-raised.
"""
import argparse
import itertools
import json
import multiprocessing as mp
import os
from datetime import datetime

parser = argparse.ArgumentParser(description="Train IQN model")
parser.add_argument("-C", "--config-file", dest="config_file", type=open, required=True,
                    help="configuration file for training parameters")
parser.add_argument("-P", "--num-procs", dest="num_procs", type=int, default=1,
                    help="number of subprocess workers to use for trial parallelization")
parser.add_argument("-D", "--device", dest="device", type=str, default="cpu",
                    help="device to run all subprocesses, could only specify 1 device in each run")


def trial_params(params):
    """Cartesian expansion of list-valued config entries (train_RL_agents.py:50-63)."""
    if isinstance(params, (str, int, float)):
        return [params]
    if isinstance(params, list):
        return params
    if isinstance(params, dict):
        keys, vals = zip(*params.items())
        return [dict(zip(keys, combo)) for combo in itertools.product(*[trial_params(v) for v in vals])]
    raise TypeError("Parameter type is incorrect.")


def params_dashboard(params):
    print("\n====== Training Setup ======\n")
    for k in ("seed", "total_timesteps", "eval_freq", "imitation_learning", "agent_type"):
        print(f"{k}: ", params[k])
    print("\n")


def run_trial(device, params):
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.envs.marinenav.env import MarineNavEnv3
    from distributional_rl_decision_and_control_amd.policy.trainer import Trainer

    exp_dir = os.path.join(params["save_dir"], "training_" + params["training_time"], "seed_" + str(params["seed"]))
    os.makedirs(exp_dir)
    with open(os.path.join(exp_dir, "trial_config.json"), "w+") as f:
        json.dump(params, f)
    train_env = MarineNavEnv3(seed=params["seed"], schedule=params["training_schedule"])
    eval_env = MarineNavEnv3(seed=253, is_eval_env=True)
    rl_agent = Agent(device=device, seed=params["seed"] + 100, agent_type=params["agent_type"])
    if "load_model" in params:
        rl_agent.load_model(params["load_model"], device)
    trainer = Trainer(train_env=train_env, eval_env=eval_env, eval_schedule=params["eval_schedule"],
                      rl_agent=rl_agent, imitation=params["imitation_learning"], il_agent=None)
    trainer.save_eval_config(exp_dir)
    trainer.learn(total_timesteps=params["total_timesteps"], eval_freq=params["eval_freq"], eval_log_path=exp_dir)


def main(argv=None):
    args = parser.parse_args(argv)
    params = json.load(args.config_file)
    params_dashboard(params)
    training_schedule = params.pop("training_schedule")
    eval_schedule = params.pop("eval_schedule")
    vectorized = params.pop("vectorized", None)
    if vectorized is not None:
        training_schedule = dict(training_schedule, vectorized=vectorized)
    trials = trial_params(params)
    timestamp = datetime.now().strftime("%Y-%m-%d-%H-%M-%S")
    for p in trials:
        p["training_time"] = timestamp
        p["training_schedule"] = training_schedule
        p["eval_schedule"] = eval_schedule
    if args.num_procs == 1:
        for p in trials:
            run_trial(args.device, p)
        return
    with mp.get_context("spawn").Pool(processes=args.num_procs) as pool:
        results = [pool.apply_async(run_trial, (args.device, p)) for p in trials]
        for r in results:
            r.get()


if __name__ == "__main__":
    main()
