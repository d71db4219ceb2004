"""Trainer -- drop-in for rfarl.policy.trainer.Trainer (trainer.py:7-410).

The single-env training loop of the reference, driving the GPU-backed MarineNavEnv3 and
Agent: same constructor, learn() cadence (learning_starts, UPDATE_EVERY, target updates,
evaluation + checkpoint at learning_starts and every eval_freq), epsilon schedule, episode
bookkeeping and printouts, evaluation metrics and the evaluations.npz / eval_configs.json
artefacts. For throughput use vec_trainer.VecTrainer (the same loop batched over envs).

Route from the unchanged reference CLI to the batched loop: the reference's run_trial passes
params["training_schedule"] straight into MarineNavEnv3 (train_RL_agents.py:85), and the reference
reads only its own keys from it (env.py:75-94). An optional "vectorized" dict in that schedule
(ignored by the reference) makes learn() drive VecTrainer instead: {"n_envs": E, "batch_size": B,
"num_tau": N, ...} are VecTrainer's keyword arguments. Evaluation, evaluations.npz and the model
files keep the reference's cadence and format; the trained networks are copied into rl_agent first.
"""
import json
import os

import numpy as np


class Trainer:
    def __init__(self, train_env, eval_env, eval_schedule, rl_agent, UPDATE_EVERY=4, learning_starts=2000,
                 target_update_interval=10000, exploration_fraction=0.25, initial_eps=0.6, final_eps=0.05,
                 imitation=False, il_agent=None, batched_eval=True):
        self.train_env = train_env
        # evaluation(): all eval configs in one device env batch (policy/batched_eval.py);
        # False runs them one by one as trainer.py:266-392 does
        self.batched_eval = batched_eval
        self.eval_env = eval_env
        self.rl_agent = rl_agent
        self.eval_config = []
        self.create_eval_configs(eval_schedule)
        self.UPDATE_EVERY = UPDATE_EVERY
        self.learning_starts = 0 if imitation else learning_starts
        self.target_update_interval = target_update_interval
        self.exploration_fraction = exploration_fraction
        self.initial_eps = initial_eps
        self.final_eps = final_eps
        self.imitation = imitation
        self.il_agent = il_agent
        if self.imitation:
            assert self.il_agent is not None, "Imitation Learning agent not given!"
        self.current_timestep = 0
        self.learning_timestep = 0
        self.eval_timesteps = []
        self.eval_observations = []
        self.eval_actions = []
        self.eval_trajectories = []
        self.eval_rewards = []
        self.eval_successes = []
        self.eval_times = []
        self.eval_energies = []
        self.eval_relations = []

    # ------------------------------------------------------------------ eval configs (trainer.py:63-83)
    def create_eval_configs(self, eval_schedule):
        self.eval_config.clear()
        env = self.eval_env
        for i, num_episode in enumerate(eval_schedule["num_episodes"]):
            for _ in range(num_episode):
                env.num_robots = eval_schedule["num_robots"][i]
                env.num_cores = eval_schedule["num_cores"][i]
                env.num_obs = eval_schedule["num_obstacles"][i]
                env.min_start_goal_dis = eval_schedule["min_start_goal_dis"][i]
                env.reset()
                self.eval_config.append(env.episode_data())

    def save_eval_config(self, directory):
        with open(os.path.join(directory, "eval_configs.json"), "w+") as f:
            json.dump(self.eval_config, f)

    # ------------------------------------------------------------------ acting helpers
    def _is_continuous(self):
        return self.rl_agent.agent_type in ("AC-IQN", "DDPG", "SAC")

    def _policy_action(self, state, eps, training):
        agent = self.rl_agent
        kind = agent.agent_type
        if training:
            if kind == "AC-IQN":
                return agent.act_ac_iqn(state, eps, use_eval=False)
            if kind == "IQN":
                return agent.act_iqn(state, eps, use_eval=False)[0]
            if kind == "Rainbow":
                return agent.act_rainbow(state, eps, use_eval=False)
            if kind == "DQN":
                return agent.act_dqn(state, eps, use_eval=False)
        else:
            if kind == "AC-IQN":
                return agent.act_ac_iqn(state)
            if kind == "IQN":
                return agent.act_iqn(state)[0]
            if kind == "Rainbow":
                return agent.act_rainbow(state)
            if kind == "DQN":
                return agent.act_dqn(state)
        raise RuntimeError("Agent type not implemented!")

    def _gather_actions(self, env, states, eps, training):
        agent = self.rl_agent
        if training and not self.imitation and agent.agent_type == "AC-IQN":
            # every active robot's act in one actor call, the same random draws in the same robot order
            # (Agent.act_ac_iqn_robots); IQN keeps per-robot calls (each draws its own quantile fractions)
            active = [i for i, rob in enumerate(env.robots) if not rob.deactivated]
            acts = agent.act_ac_iqn_robots([states[i] for i in active], eps, use_eval=False)
            actions = [None] * len(env.robots)
            for i, a in zip(active, acts):
                actions[i] = a
            return actions
        actions = []
        for i, rob in enumerate(env.robots):
            if rob.deactivated:
                actions.append(None)
            elif training and self.imitation:
                actions.append(self.il_agent.act(states[i]))
            else:
                actions.append(self._policy_action(states[i], eps, training))
        return actions

    # ------------------------------------------------------------------ training loop (trainer.py:85-255)
    def learn(self, total_timesteps, eval_freq, eval_log_path, verbose=True):
        sched = getattr(self.train_env, "schedule", None)
        if isinstance(sched, dict) and sched.get("vectorized") is not None:
            return self.learn_vectorized(sched["vectorized"], total_timesteps, eval_freq, eval_log_path, verbose)
        agent = self.rl_agent
        env = self.train_env
        states, _, _ = env.reset()
        ep = self._new_episode(len(env.robots))
        eps = None
        while self.current_timestep <= total_timesteps:
            if not self.imitation:
                eps = self.linear_eps(total_timesteps)
            actions = self._gather_actions(env, states, eps, training=True)
            next_states, rewards, dones, infos = env.step(actions, self._is_continuous())
            self._record_transitions(env, ep, states, actions, rewards, next_states, dones)
            end_episode = (ep["length"] >= 1000) or env.check_all_deactivated()
            if self.current_timestep >= self.learning_starts:
                if not agent.training:
                    continue
                self._learning_phase(eval_freq, eval_log_path)
            if end_episode:
                ep["num"] += 1
                if verbose:
                    self._print_episode(ep, eps, infos, total_timesteps)
                states, _, _ = env.reset()
                ep = self._new_episode(len(env.robots), ep["num"])
            else:
                states = next_states
                ep["length"] += 1
            self.current_timestep += 1

    def learn_vectorized(self, vec, total_timesteps, eval_freq, eval_log_path, verbose=True):
        """learn() on the batched GPU loop (vec_trainer.VecTrainer): one iteration advances every env of
        the batch by one step (E env-steps) and runs one learn step of batch B. Evaluation and the
        checkpoint happen at the first learning iteration and whenever the env-step count crosses a
        multiple of eval_freq (trainer.py:200-206), with rl_agent holding the trained networks."""
        import torch

        from ..vec_trainer import VecTrainer
        agent = self.rl_agent
        if agent.agent_type not in ("AC-IQN", "IQN", "Rainbow"):
            raise ValueError(f"vectorized training covers AC-IQN, IQN and Rainbow, not {agent.agent_type}")
        sched = {k: v for k, v in self.train_env.schedule.items() if k != "vectorized"}
        kw = dict(vec)
        kw.setdefault("graphs", True)
        for key, sk in (("num_robots", "num_robots"), ("num_obs", "num_obstacles"), ("num_cores", "num_cores")):
            if sk in sched:
                kw.setdefault(key, max(sched[sk]))
        # the Trainer's cadence in the batched loop's units: learning starts once the replay holds
        # learning_starts transitions (and at least one batch); the hard target update every
        # target_update_interval env-steps = every target_update_interval / UPDATE_EVERY learn steps
        # (trainer.py:175-192: one B=64 learn step per UPDATE_EVERY timesteps)
        kw.setdefault("learning_starts", max(int(kw.get("batch_size", 4096)), int(self.learning_starts)))
        kw.setdefault("target_update_interval", max(1, int(self.target_update_interval) // int(self.UPDATE_EVERY)))
        tr = VecTrainer(agent_type=agent.agent_type, seed=getattr(self.train_env, "seed", 0), device=agent.device,
                        total_timesteps=total_timesteps, schedule=sched, gamma=agent.GAMMA, lr=agent.LR,
                        exploration_fraction=self.exploration_fraction, initial_eps=self.initial_eps,
                        final_eps=self.final_eps, **kw)
        # start from rl_agent's networks (its seeded init, or what load_model put there), not the
        # batched trainer's own initialisation
        tr.load_policies(agent.policy_local, agent.policy_target)
        self.vec_trainer = tr
        next_eval = None
        while self.current_timestep < total_timesteps:   # iteration k covers env-steps [kE, (k + 1)E)
            tr.env.apply_schedule(tr.env.total_timesteps)
            learning = tr.replay_size_host() >= tr.learning_starts
            tr.iteration()
            self.current_timestep += tr.E
            if learning and (next_eval is None or self.current_timestep >= next_eval):
                next_eval = (self.current_timestep // eval_freq + 1) * eval_freq
                self._sync_agent(tr)
                self.evaluation()
                self.save_evaluation(eval_log_path)
                if agent.training:
                    agent.save_latest_model(eval_log_path)
                if verbose:
                    st = tr.env.episode_stats()
                    print(f"timesteps {self.current_timestep}/{total_timesteps}: {st}")
        torch.cuda.synchronize(tr.device)
        self._sync_agent(tr)
        return tr

    def _sync_agent(self, tr):
        """rl_agent's local / target networks <- the batched trainer's (same architectures)."""
        import torch
        pairs = [(self.rl_agent.policy_local, tr.local), (self.rl_agent.policy_target, tr.target)]
        with torch.no_grad():
            for dst, src in pairs:
                if hasattr(src, "actor"):   # AC_IQN_Policy holds two modules
                    dst.actor.load_state_dict(src.actor.state_dict())
                    dst.critic.load_state_dict(src.critic.state_dict())
                else:
                    dst.load_state_dict(src.state_dict())
        if hasattr(self.rl_agent, "_fused"):
            self.rl_agent._fused = None   # the drop-in learner re-packs its weight images on its next train()

    @staticmethod
    def _new_episode(n, num=0):
        return {"rewards": np.zeros(n), "deactivated_t": [-1] * n, "length": 0, "num": num}

    def _record_transitions(self, env, ep, states, actions, rewards, next_states, dones):
        agent = self.rl_agent
        for i, rob in enumerate(env.robots):
            if rob.deactivated:
                continue
            ep["rewards"][i] += agent.GAMMA ** ep["length"] * rewards[i]
            if agent.training:
                if agent.agent_type == "Rainbow":
                    agent.memory.append(states[i], actions[i], rewards[i], dones[i])
                else:
                    agent.memory.add((states[i], actions[i], rewards[i], next_states[i], dones[i]))
            if rob.collision or rob.reach_goal:
                rob.deactivated = True
                ep["deactivated_t"][i] = ep["length"]

    def _learning_phase(self, eval_freq, eval_log_path):
        agent = self.rl_agent
        t = self.current_timestep
        if t % self.UPDATE_EVERY == 0:
            n = agent.memory.transitions.num_elements() if agent.agent_type == "Rainbow" else agent.memory.size()
            if n > agent.BATCH_SIZE:
                agent.train()
        if t % self.target_update_interval == 0:
            agent.soft_update()
        if t == self.learning_starts or t % eval_freq == 0:
            self.evaluation()
            self.save_evaluation(eval_log_path)
            if agent.training:
                agent.save_latest_model(eval_log_path)

    def _print_episode(self, ep, eps, infos, total_timesteps):
        print("======== IL Episode Info ========" if self.imitation else "======== RL Episode Info ========")
        print("current ep_length: ", ep["length"])
        print("current ep_num: ", ep["num"])
        if not self.imitation:
            print("current exploration rate: ", eps)
        print("current timesteps: ", self.current_timestep)
        print("total timesteps: ", total_timesteps)
        print("======== Episode Info ========\n")
        print("======== Robots Info ========")
        for i in range(len(self.train_env.robots)):
            info = infos[i]["state"]
            if info in ("deactivated after collision", "deactivated after reaching goal"):
                print(f"Robot {i} ep reward: {ep['rewards'][i]:.2f}, {info} at step {ep['deactivated_t'][i]}")
            else:
                print(f"Robot {i} ep reward: {ep['rewards'][i]:.2f}, {info}")
        print("======== Robots Info ========\n")

    def linear_eps(self, total_timesteps):  # trainer.py:257-264
        progress = self.current_timestep / total_timesteps
        if progress < self.exploration_fraction:
            r = progress / self.exploration_fraction
            return self.initial_eps + r * (self.final_eps - self.initial_eps)
        return self.final_eps

    # ------------------------------------------------------------------ evaluation (trainer.py:266-410)
    def _run_eval_episode(self, config):
        env = self.eval_env
        agent = self.rl_agent
        state, _, _ = env.reset_with_eval_config(config)
        n = len(env.robots)
        rewards, times, energies = [0.0] * n, [0.0] * n, [0.0] * n
        length = 0
        end_episode = False
        while not end_episode:
            action = self._gather_actions(env, state, 0.0, training=False)
            state, reward, done, info = env.step(action, self._is_continuous())
            for i, rob in enumerate(env.robots):
                if rob.deactivated:
                    continue
                rewards[i] += agent.GAMMA ** length * reward[i]
                times[i] += rob.dt * rob.N
                energies[i] += rob.compute_step_energy_cost()
                if rob.collision or rob.reach_goal:
                    rob.deactivated = True
            end_episode = (length >= 1000) or env.check_any_collision() or env.check_all_deactivated()
            length += 1
        histories = ([rob.observation_history for rob in env.robots], [rob.action_history for rob in env.robots],
                     [rob.trajectory for rob in env.robots])
        import copy
        return (copy.deepcopy(histories), np.mean(rewards), bool(env.check_all_reach_goal()), np.mean(times),
                np.mean(energies), [[] for _ in range(n)])

    def evaluation(self, batched=None):
        batched = self.batched_eval if batched is None else batched
        if batched:
            from .batched_eval import evaluate_configs
            print(f"Evaluating episodes 0-{len(self.eval_config) - 1} (one batch)")
            res = evaluate_configs(self.rl_agent, self.eval_config, template_env=self.eval_env)
            obs_d, act_d, traj_d = res["observations"], res["actions"], res["trajectories"]
            rew_d, succ_d, time_d, en_d, rel_d = (res["rewards"], res["successes"], res["times"], res["energies"],
                                                  res["relations"])
        else:
            obs_d, act_d, traj_d, rew_d, succ_d, time_d, en_d, rel_d = [], [], [], [], [], [], [], []
            for idx, config in enumerate(self.eval_config):
                print(f"Evaluating episode {idx}")
                (obs, acts, trajs), r, s, t, e, rel = self._run_eval_episode(config)
                obs_d.append(obs)
                act_d.append(acts)
                traj_d.append(trajs)
                rew_d.append(r)
                succ_d.append(s)
                time_d.append(t)
                en_d.append(e)
                rel_d.append(rel)
        avg_r = np.mean(rew_d)
        success_rate = np.sum(succ_d) / len(succ_d)
        idx = np.where(np.array(succ_d) == 1)[0]
        avg_t = None if np.shape(idx)[0] == 0 else np.mean(np.array(time_d)[idx])
        avg_e = None if np.shape(idx)[0] == 0 else np.mean(np.array(en_d)[idx])
        print("++++++++ Evaluation Info ++++++++")
        print(f"Avg cumulative reward: {avg_r:.2f}")
        print(f"Success rate: {success_rate:.2f}")
        if avg_t is not None:
            print(f"Avg time: {avg_t:.2f}")
            print(f"Avg energy: {avg_e:.2f}")
        print("++++++++ Evaluation Info ++++++++\n")
        self.eval_timesteps.append(self.current_timestep)
        self.eval_observations.append(obs_d)
        self.eval_actions.append(act_d)
        self.eval_trajectories.append(traj_d)
        self.eval_rewards.append(rew_d)
        self.eval_successes.append(succ_d)
        self.eval_times.append(time_d)
        self.eval_energies.append(en_d)
        self.eval_relations.append(rel_d)

    def save_evaluation(self, eval_log_path):
        fields = dict(timesteps=self.eval_timesteps, observations=self.eval_observations, actions=self.eval_actions,
                      trajectories=self.eval_trajectories, rewards=self.eval_rewards, successes=self.eval_successes,
                      times=self.eval_times, energies=self.eval_energies, relations=self.eval_relations)
        arrays = {k: np.array(v, dtype=object) for k, v in fields.items()}  # trainer.py:397-410 format
        np.savez(os.path.join(eval_log_path, "evaluations.npz"), **arrays)
