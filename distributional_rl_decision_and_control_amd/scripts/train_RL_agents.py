"""train_RL_agents -- the reference CLI (rfarl/rfarl/scripts/train_RL_agents.py:1-141) on
the GPU-backed env/agent/trainer.

    python -m distributional_rl_decision_and_control_amd.scripts.train_RL_agents -C config/ac_iqn.json [-P n] [-D dev]

Same flags, the same config JSON schema (list-valued keys expand to a cartesian product of
trials), the same per-trial directory layout and artefacts. Optional extra keys, ignored by
the reference: "vectorized": {"n_envs": E, ...} runs the batched VecTrainer instead.
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
    if "vectorized" in params:
        return run_vectorized(device, params, exp_dir)
    train_env = MarineNavEnv3(seed=params["seed"], schedule=params["training_schedule"])
    eval_env = MarineNavEnv3(seed=253, is_eval_env=True)
    rl_agent = Agent(device=device, seed=params["seed"] + 100, agent_type=params["agent_type"])
    if "load_model" in params:
        rl_agent.load_model(params["load_model"], device)
    trainer = Trainer(train_env=train_env, eval_env=eval_env, eval_schedule=params["eval_schedule"],
                      rl_agent=rl_agent, imitation=params["imitation_learning"], il_agent=None)
    trainer.save_eval_config(exp_dir)
    trainer.learn(total_timesteps=params["total_timesteps"], eval_freq=params["eval_freq"], eval_log_path=exp_dir)


def run_vectorized(device, params, exp_dir):
    import torch
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    v = dict(params["vectorized"])
    dev = torch.device("cuda") if device in (None, "cpu") else torch.device(device)
    tr = VecTrainer(agent_type=params["agent_type"], seed=params["seed"], device=dev,
                    total_timesteps=params["total_timesteps"], schedule=params.get("training_schedule"), **v)
    iters = max(1, params["total_timesteps"] // tr.E)
    for k in range(iters):
        tr.env.apply_schedule(tr.env.total_timesteps)
        tr.iteration()
        if (k + 1) % max(1, iters // 10) == 0:
            print(f"iteration {k + 1}/{iters}: {tr.env.episode_stats()}")
    tr.local.save(exp_dir) if hasattr(tr.local, "save") else None


def main(argv=None):
    args = parser.parse_args(argv)
    params = json.load(args.config_file)
    params_dashboard(params)
    training_schedule = params.pop("training_schedule")
    eval_schedule = params.pop("eval_schedule")
    vectorized = params.pop("vectorized", None)
    trials = trial_params(params)
    timestamp = datetime.now().strftime("%Y-%m-%d-%H-%M-%S")
    for p in trials:
        p["training_time"] = timestamp
        p["training_schedule"] = training_schedule
        p["eval_schedule"] = eval_schedule
        if vectorized is not None:
            p["vectorized"] = vectorized
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
