"""Trainer.evaluation (trainer.py:266-392) with every evaluation config in one device env batch.

The reference runs its eval configs one after another, one robot at a time (a batch-1 network
call per robot per step). Here all configs advance together:

  * the envs are the drop-in MarineNavEnv3 instances, each reset from its config
    (reset_with_eval_config, env.py:503-610), so every robot keeps its own seeded RandomState;
  * per step, ONE batched greedy policy call over every active robot of every running episode
    (act_ac_iqn / act_iqn / act_rainbow with eps = 0, agent.py:207-250,308-324). Each robot still
    consumes its one `random.random()` draw, so Python's global RNG ends where the sequential
    evaluation leaves it;
  * ONE asvrl_env_step launch for all running envs (envs.marinenav.env.run_env_step; envs are
    grouped by parameter set, since a launch takes one), with every robot's perception noise
    drawn from its own RandomState in the reference's order;
  * the per-robot bookkeeping of trainer.py:331-345 (discounted return, time dt*N, energy from
    Robot.compute_step_energy_cost, deactivation, episode end on timeout / any collision / all
    deactivated) and the per-config metrics of trainer.py:347-365, unchanged.

Results equal the sequential evaluation up to the rounding of a batched vs batch-1 GEMM in the
policy (tests/test_batched_eval_gpu.py); IQN draws its K = 32 quantile fractions per call, so
its two paths agree in distribution only, as two sequential runs would.
"""
import copy
import random

import numpy as np
import torch

from ..device_env import DeviceEnvBatch
from ..envs.marinenav.env import MarineNavEnv3, run_env_step


def _params_key(env):
    """The env-level launch parameters (envs sharing them share a launch; robots with their own vehicle /
    perception parameters go through the per-robot table, envs.marinenav.env.set_batch_params)."""
    return env.env_key()


@torch.no_grad()
def batched_greedy_actions(agent, states, taus=None):
    """Greedy actions (eps = 0) for a list of per-robot states in one network call. Each robot
    consumes one random.random() like the batch-1 act functions; the (probability ~2^-53) draw
    that is not > 0 explores as they do. taus (IQN only): the K quantile fractions of every row
    ((n, K) or (n, K, 1)) instead of fresh draws -- act_iqn's calc_cos draws (IQN_model.py:56-72),
    injected by the parity test."""
    kind = agent.agent_type
    s = agent.state_to_tensor(agent.memory.state_batch(states))
    if kind == "AC-IQN":
        net = agent.policy_local.actor
        net.eval()
        a = net(s).float().cpu().numpy()
        net.train()
        greedy = [a[i].tolist() for i in range(len(states))]
    elif kind == "IQN":
        net = agent.policy_local
        net.eval()
        q, _ = net(s, net.K, 1.0, taus=taus)
        net.train()
        greedy = [int(v) for v in q.mean(dim=1).argmax(dim=1).cpu().numpy()]
    elif kind == "Rainbow":
        net = agent.policy_local
        net.eval()
        p = net(s)
        net.train()
        greedy = [int(v) for v in (p * agent.support).sum(2).argmax(1).cpu().numpy()]
    elif kind == "DQN":
        net = agent.policy_local
        net.eval()
        q = net(s)
        net.train()
        greedy = [int(v) for v in q.argmax(dim=1).cpu().numpy()]
    else:
        raise RuntimeError("Agent type not implemented!")
    out = []
    for g in greedy:
        if random.random() > 0.0:
            out.append(g)
        elif kind == "AC-IQN":
            out.append([np.random.uniform(low=lo, high=hi) for lo, hi in agent.value_ranges_of_action])
        else:
            out.append(random.choice(np.arange(agent.action_size)))
    return out


def evaluate_configs(agent, configs, device=None, template_env=None, policy=None):
    """Run every eval config to its end in one batch. Returns the per-config lists
    (observations, actions, trajectories, rewards, successes, times, energies, relations) of
    trainer.py:347-365. `policy(rows, states, length)` replaces the greedy policy call (rows: the (config,
    robot) pairs that act this step, states: their states, length: each config's step count); the default
    is batched_greedy_actions. The parity tests use it to replay recorded actions (teacher forcing)."""
    E = len(configs)
    dev = torch.device(device) if device is not None else (template_env._device if template_env is not None
                                                           else torch.device("cuda"))
    envs = []
    states = []
    for cfg in configs:
        env = MarineNavEnv3(seed=0, is_eval_env=True, device=dev)
        if template_env is not None:
            # reset_with_eval_config seeds each robot with rd.randint(0, 5 * num_robots) using the
            # eval env's CURRENT curriculum attributes (env.py:569), not the config's
            for k in ("num_robots", "num_cores", "num_obs", "min_start_goal_dis"):
                setattr(env, k, getattr(template_env, k))
        st, _, _ = env.reset_with_eval_config(cfg)
        envs.append(env)
        states.append(st)
    continuous = agent.agent_type in ("AC-IQN", "DDPG", "SAC")
    n = [len(env.robots) for env in envs]
    rewards = [[0.0] * k for k in n]
    times = [[0.0] * k for k in n]
    energies = [[0.0] * k for k in n]
    length = [0] * E
    running = list(range(E))
    groups = {}
    for e in range(E):
        groups.setdefault(_params_key(envs[e]), []).append(e)
    batches = {}
    for key, members in groups.items():
        R = max(len(envs[e].robots) for e in members)
        O = max(len(envs[e].obstacles) for e in members)
        Cm = max(len(envs[e].cores) for e in members)
        batches[key] = DeviceEnvBatch(len(members), max(R, 1), max(O, 1), max(Cm, 1), device=dev, obs64=True)
    while running:
        # one policy call for every active robot of every running episode (trainer.py:300-322)
        rows = [(e, i) for e in running for i, rob in enumerate(envs[e].robots) if not rob.deactivated]
        st = [states[e][i] for e, i in rows]
        if policy is not None:
            acts = policy(rows, st, length) if rows else []
        else:
            acts = batched_greedy_actions(agent, st) if rows else []
        actions = {e: [None] * n[e] for e in running}
        for (e, i), a in zip(rows, acts):
            actions[e][i] = a
        # one env-step launch per parameter group (trainer.py:329)
        results = {}
        for key, members in groups.items():
            live = [e for e in members if e in actions]
            if not live:
                continue
            for e in live:
                env = envs[e]
                assert env.check_all_reach_goal() is not True, "All robots reach goals, not actions are available!"
            active = {e: [not rob.deactivated for rob in envs[e].robots] for e in live}
            outs = run_env_step(batches[key], [envs[e] for e in live], [actions[e] for e in live], continuous, True)
            for e, out in zip(live, outs):
                results[e] = envs[e]._finish_step(actions[e], active[e], out)
        still = []
        for e in running:
            env = envs[e]
            states[e], reward, _, _ = results[e]
            for i, rob in enumerate(env.robots):   # trainer.py:331-339
                if rob.deactivated:
                    continue
                rewards[e][i] += agent.GAMMA ** length[e] * reward[i]
                times[e][i] += rob.dt * rob.N
                energies[e][i] += rob.compute_step_energy_cost()
                if rob.collision or rob.reach_goal:
                    rob.deactivated = True
            end_episode = (length[e] >= 1000) or env.check_any_collision() or env.check_all_deactivated()
            length[e] += 1
            if not end_episode:
                still.append(e)
        running = still
    out = dict(observations=[], actions=[], trajectories=[], rewards=[], successes=[], times=[], energies=[],
               relations=[])
    for e, env in enumerate(envs):   # trainer.py:347-365
        out["observations"].append(copy.deepcopy([rob.observation_history for rob in env.robots]))
        out["actions"].append(copy.deepcopy([rob.action_history for rob in env.robots]))
        out["trajectories"].append(copy.deepcopy([rob.trajectory for rob in env.robots]))
        out["rewards"].append(np.mean(rewards[e]))
        out["successes"].append(bool(env.check_all_reach_goal()))
        out["times"].append(np.mean(times[e]))
        out["energies"].append(np.mean(energies[e]))
        out["relations"].append([[] for _ in range(n[e])])
    out["lengths"] = length
    return out
