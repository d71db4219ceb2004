"""VecTrainer -- the fused rollout + learn loop of rfarl's Trainer.learn (trainer.py:85-255),
batched over E envs on one GPU, data-parallel over ranks.

One iteration (= one `step` of bench.py):
  1. act: the local actor on every robot of every env (E*R rows), epsilon-greedy on device
     (trainer.py:106-135, agent.py:207-225; linear epsilon schedule trainer.py:257-264)
  2. env step kernel with the trainer bookkeeping fused (asvrl_env_step)
  3. replay push of the transitions of robots that acted (asvrl_replay_push, trainer.py:157-166)
  4. device reset of finished envs + their first observation (asvrl_env_reset, trainer.py:212-245)
  5. learn: sample B transitions (asvrl_replay_sample) and one distributional update
     (AC-IQN: two dependent optimizer steps, critic then actor; IQN: one)
  6. hard target update every `target_update_interval` learn steps (agent.py:643-679, TAU=1)

Cadence in the batched setting: one learn step of batch B per iteration (after
`learning_starts` transitions) replaces the reference's one B=64 step per 4 single-env
timesteps; target updates count learn steps (2500 = 10000 timesteps / UPDATE_EVERY 4).
With `graphs=True` steps 1-5 are captured once into a HIP graph and replayed.
"""
import os
import time

import torch

from . import streams
from .fused_critic import FusedACIQN, ac_iqn_update_fused, fused_supported
from .fused_update import FusedACIQNState, ac_iqn_update_fused2
from .fused_iqn import FusedIQNState, iqn_update_fused
from .fused_iqn import supported as fused_iqn_supported
from .fused_rainbow import FusedRainbow
from .fused_update import supported as fused2_supported
from .learn_ops import DevicePER, DeviceReplay, split_rows
from .learner import FlatGrads, FusedAdam, GradSync, ac_iqn_update, iqn_update, rainbow_update, rainbow_update_rows
from .policy.AC_IQN_model import AC_IQN_Policy
from .policy.IQN_model import IQN_Policy
from .policy.Rainbow_model import Rainbow_Policy
from .vec_env import VecMarineNavEnv, split_obs

DEFAULT_NET = dict(self_dimension=7, object_dimension=5, max_object_num=5, self_feature_dimension=56,
                   object_feature_dimension=40, concat_feature_dimension=256, hidden_dimension=128)


class VecTrainer:
    def __init__(self, n_envs=4096, agent_type="AC-IQN", num_robots=5, num_obs=4, num_cores=0, min_start_goal_dis=40.0,
                 width=55.0, batch_size=4096, num_tau=32, buffer_size=4_000_000, lr=1e-4, gamma=0.99,
                 learning_starts=None, target_update_interval=2500, total_timesteps=6_000_000,
                 exploration_fraction=0.25, initial_eps=0.6, final_eps=0.05, amp_dtype=torch.bfloat16, seed=0,
                 device="cuda", sync=None, graphs=False, schedule=None, net_seed=100, fused=True,
                 fused_adam=True, overlap=True, unroll=1, pipeline=False, chain=None):
        self.device = torch.device(device)
        self.agent_type = agent_type
        self.continuous = agent_type == "AC-IQN"
        self.env = VecMarineNavEnv(n_envs, num_robots, num_obs, num_cores, min_start_goal_dis, width, seed=seed,
                                   device=self.device, is_continuous=self.continuous, gamma=gamma, schedule=schedule)
        self.E, self.R = n_envs, self.env.max_robots
        self.B, self.num_tau, self.gamma = batch_size, num_tau, gamma
        self.amp_dtype = amp_dtype
        self.sync = sync
        self.seed = seed
        self.target_update_interval = target_update_interval
        self.total_timesteps = total_timesteps
        self.exploration_fraction, self.initial_eps, self.final_eps = exploration_fraction, initial_eps, final_eps
        self.learning_starts = learning_starts if learning_starts is not None else batch_size
        capturable = bool(graphs)
        self.fused = self.fused2 = self.fused_iqn = self.fused_rb = None
        if agent_type == "AC-IQN":
            self.local = AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1.0, 1.0], [-1.0, 1.0]],
                                       device=self.device, seed=net_seed)
            self.target = AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1.0, 1.0], [-1.0, 1.0]],
                                        device=self.device, seed=net_seed)
            for p in list(self.target.actor.parameters()) + list(self.target.critic.parameters()):
                p.requires_grad_(False)
            if fused_adam:
                # clip + Adam as two kernels over flat buffers (must precede FusedACIQN's packs)
                self.actor_opt = FusedAdam(self.local.actor.parameters(), lr=lr)
                self.critic_opt = FusedAdam(self.local.critic.parameters(), lr=lr)
                self.actor_grads, self.critic_grads = self.actor_opt.grads, self.critic_opt.grads
            else:
                self.critic_grads = FlatGrads(self.local.critic.parameters())
                self.actor_grads = FlatGrads(self.local.actor.parameters())
                self.actor_opt = torch.optim.Adam(self.local.actor.parameters(), lr=lr, capturable=capturable)
                self.critic_opt = torch.optim.Adam(self.local.critic.parameters(), lr=lr, capturable=capturable)
            self.action_dim = 2
            # fused=True: the whole update on hand-written kernels (fused_update.py, needs the fused
            # optimiser); "v1": only the critic trunk fused; False: torch
            if fused is True and fused_adam and amp_dtype is not None and fused2_supported(self.local, batch_size,
                                                                                          num_tau):
                self.fused2 = FusedACIQNState(self.local, self.target, batch_size, num_tau)
            elif fused and amp_dtype is not None and fused_supported(self.local.critic, batch_size, num_tau):
                self.fused = FusedACIQN(self.local, self.target, batch_size, num_tau)
        elif agent_type == "IQN":
            self.local = IQN_Policy(**DEFAULT_NET, action_size=25, device=self.device, seed=net_seed).to(self.device)
            self.target = IQN_Policy(**DEFAULT_NET, action_size=25, device=self.device, seed=net_seed).to(self.device)
            for p in self.target.parameters():
                p.requires_grad_(False)
            if fused_adam:
                self.opt = FusedAdam(self.local.parameters(), lr=lr)
                self.grads = self.opt.grads
            else:
                self.grads = FlatGrads(self.local.parameters())
                self.opt = torch.optim.Adam(self.local.parameters(), lr=lr, capturable=capturable)
            self.action_dim = 1
            # fused=True: the whole IQN update and act_iqn on hand-written kernels (fused_iqn.py)
            if fused is True and fused_adam and amp_dtype is not None and fused_iqn_supported(self.local, batch_size,
                                                                                            num_tau):
                self.fused_iqn = FusedIQNState(self.local, self.target, batch_size, num_tau)
        elif agent_type == "Rainbow":
            # Rainbow_Policy (dueling NoisyNet C51, 51 atoms on [-1, 1]) with the prioritised n-step
            # replay in HBM, one stream per robot (agent.py:597-641, replay_memory_rainbow.py)
            self.local = Rainbow_Policy(**DEFAULT_NET, action_size=25, atoms=51, device=self.device,
                                        seed=net_seed).to(self.device)
            self.target = Rainbow_Policy(**DEFAULT_NET, action_size=25, atoms=51, device=self.device,
                                         seed=net_seed).to(self.device)
            for p in self.target.parameters():
                p.requires_grad_(False)
            if fused_adam:
                self.opt = FusedAdam(self.local.parameters(), lr=lr)
                self.grads = self.opt.grads
            else:
                self.grads = FlatGrads(self.local.parameters())
                self.opt = torch.optim.Adam(self.local.parameters(), lr=lr, capturable=capturable)
            self.action_dim = 1
            self.n_step = 3
            self.support = torch.linspace(-1.0, 1.0, 51, device=self.device)
            # one online forward over s and s_{t+n} (learner.rainbow_update_rows) or two (rainbow_update)
            self.rainbow_packed = os.environ.get("ASVRL_RAINBOW_PACKED", "0") == "1"
            # fused=True: noisy weights, dueling head, loss gradient and act on hand-written kernels
            # (fused_rainbow.py; fp32 GEMMs); otherwise the torch update with the C51 kernel
            if fused is True and fused_adam:
                self.fused_rb = FusedRainbow(self.local, self.target, batch_size, self.support)
        else:
            raise NotImplementedError(f"VecTrainer agent_type {agent_type!r} (AC-IQN, IQN and Rainbow are batched)")
        NT = self.E * self.R
        self.per = None
        if agent_type == "Rainbow":
            slots = max(min(buffer_size, 1 << 22) // NT, self.n_step + 3)
            self.per = DevicePER(slots * NT, stride=NT, n_step=self.n_step, discount=gamma, deferred=True,
                                 device=self.device)
            self.replay = None
            self.per_idx = torch.zeros(self.B, dtype=torch.int64, device=self.device)
            # the tree holds complete windows once n + 1 pushes are in
            self.learning_starts = max(self.learning_starts, (self.n_step + 1) * NT + self.B)
        else:
            self.replay = DeviceReplay(max(buffer_size, 2 * NT), device=self.device)
        self.actions = torch.zeros((NT, 2), dtype=torch.float64, device=self.device)
        self.learn_counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.batch_rows = torch.zeros((self.B, 88), dtype=torch.float32, device=self.device)
        # the fused updates' quantile fractions (AC-IQN: target, local, actor step; IQN: the first two)
        self.taus = torch.zeros((3, self.B, self.num_tau), dtype=torch.float32, device=self.device)
        # pipelined AC-IQN learner (opt-in): the next batch and its target quantiles are produced
        # beside the current actor step (fused_update.target_q), so the critic step starts at once.
        # Two buffer sets alternate by parity; a captured graph then holds two iterations (one per
        # parity), on the joined schedule. Measured: no gain at the bench shape (0.5595 vs 0.559 ms) --
        # the GPU is saturated, the overlap only moves the contention. A chained form (the batch sampled
        # against the snapshot behind the previous push) was bit-identical and 11 % slower
        # (profiles/r02_pipeline_chain_ab.txt), and its graph segfaulted in hipGraphLaunch late in the
        # full GPU suite (never alone): reverted.
        self.pipeline = bool(pipeline) and self.fused2 is not None
        if self.pipeline:
            self.rows_buf = [self.batch_rows, torch.zeros_like(self.batch_rows)]
            self.taus_buf = [self.taus, torch.zeros_like(self.taus)]
            self._parity = 0
            self._primed = False
        self.learn_steps = 0
        self.iterations = 0
        self.last_losses = None
        self.graphs = graphs
        self._graph = None
        # iterations per captured graph: one replay enqueues `unroll` whole iterations (the host
        # calls iteration() once per iteration; every unroll-th call replays). Measured: 2 gives no
        # gain over 1 (0.564 vs 0.559 ms/step), the in-graph joins keep the same gaps
        self.unroll = max(1, int(unroll), 2 if self.pipeline and graphs else 1)
        self._phase = 0
        self._graph_learn = None
        # rollout / learn on two streams (fused learners): the learner samples against a
        # snapshot of the ring state taken before this iteration's push, skipping the oldest
        # E*R entries the push may overwrite, and waits for the act kernel before the actor
        # weights change
        self.overlap = bool(overlap)
        self.ring_snap = torch.zeros(2, dtype=torch.int64, device=self.device)
        self._streams = None
        # inside a captured graph of an even number of iterations, the two streams are ordered by the
        # exact dependencies instead of a join per iteration: act(i) after learn(i-1) (new weights),
        # learn(i) after the snapshot of the ring taken right behind push(i-1) (double-buffered, the
        # same state the joined schedule samples against), learn(i)'s weight updates after act(i).
        # Same operations on the same data as the joined schedule (tested bit for bit); the next
        # learner no longer waits for the rollout's tail (reset, observation pass, copies). chain=None:
        # AC-IQN only (measured 0.346 -> 0.340 ms/step; IQN, whose act kernel fills the GPU, 0.363 ->
        # 0.366: profiles/r02_chain_schedule_ab.txt)
        self.chain = (agent_type == "AC-IQN") if chain is None else bool(chain)
        self.ring_snap2 = torch.zeros((2, 2), dtype=torch.int64, device=self.device)
        self._gen = torch.Generator(device=self.device)
        self._gen.manual_seed(seed + 12345)
        self.env.reset()

    # ------------------------------------------------------------------ pieces
    def epsilon(self):
        """trainer.py:257-264 as a device scalar of the device step counter (graph-safe)."""
        steps = self.env.counter.to(torch.float32) * float(self.E)
        progress = steps / float(self.total_timesteps)
        r = progress / self.exploration_fraction
        eps = self.initial_eps + r * (self.final_eps - self.initial_eps)
        return torch.where(progress < self.exploration_fraction, eps, torch.full_like(eps, self.final_eps))

    @torch.no_grad()
    def act(self):
        if self.fused_rb is not None:
            # composed noisy weights, logits, one head kernel: expected Q, argmax, epsilon-greedy
            self.fused_rb.act(self.env.obs_cur, self.actions, self.env.counter, self.E, self.total_timesteps,
                              self.exploration_fraction, self.initial_eps, self.final_eps, self.seed + 4242)
            return
        if self.fused_iqn is not None:
            # encoders + one kernel: K = 32 quantiles per robot, mean, argmax, epsilon-greedy
            self.fused_iqn.act(self.env.obs_cur, self.actions, self.env.counter, self.E, self.total_timesteps,
                               self.exploration_fraction, self.initial_eps, self.final_eps, self.seed + 4242)
            return
        if self.fused2 is not None:
            # one kernel: actor on every robot row + epsilon-greedy on the device step counter
            self.fused2.act(self.env.obs_cur, self.actions, self.env.counter, self.E, self.total_timesteps,
                            self.exploration_fraction, self.initial_eps, self.final_eps, self.seed + 4242)
            return
        obs = split_obs(self.env.obs_cur)
        NT = obs[0].shape[0]
        eps = self.epsilon()
        explore = torch.rand((NT, 1), device=self.device) < eps
        if self.agent_type == "Rainbow":
            # act_rainbow (agent.py:308-324) on every robot row, training-mode noisy weights
            amp = torch.autocast("cuda", dtype=self.amp_dtype) if self.amp_dtype is not None else _null()
            with amp:
                p = self.local(obs)
            greedy = (p.float() * self.support).sum(2).argmax(1)
            rnd = torch.randint(0, 25, (NT,), device=self.device)
            self.actions[:, 0].copy_(torch.where(explore.squeeze(1), rnd, greedy))
            return
        if self.agent_type == "AC-IQN":
            # fp32 actor when the critic is fused (see ac_iqn_update_fused)
            use_amp = self.amp_dtype is not None and self.fused is None
            amp = torch.autocast("cuda", dtype=self.amp_dtype) if use_amp else _null()
            with amp:
                a = self.local.actor(obs).float()
            rnd = torch.rand((NT, 2), device=self.device) * 2.0 - 1.0
            self.actions.copy_(torch.where(explore, rnd, a))
        else:
            amp = torch.autocast("cuda", dtype=self.amp_dtype) if self.amp_dtype is not None else _null()
            with amp:
                q, _ = self.local(obs, self.local.K)
            greedy = q.float().mean(dim=1).argmax(dim=1)
            rnd = torch.randint(0, 25, (NT,), device=self.device)
            self.actions[:, 0].copy_(torch.where(explore.squeeze(1), rnd, greedy))

    def _fused_learner(self):
        return self.fused2 is not None or self.fused_iqn is not None

    def _push(self):
        env = self.env
        if self.per is not None:   # ReplayMemory.append of every robot that acted (trainer.py:163-164)
            self.per.push(env.obs_cur, env.cnt_next, self.actions[:, :1], env.batch.reward, env.batch.done)
            return
        self.replay.push(env.obs_cur, env.obs_next, env.cnt_next, self.actions[:, :self.action_dim].contiguous()
                         if self.action_dim == 1 else self.actions, env.batch.reward, env.batch.done)

    def rollout(self):
        self.act()
        self.env.step(self.actions)
        self._push()
        self.env.auto_reset()

    def _produce(self, nxt, state, guard, counter):
        st = self.fused2
        rows = self.replay.sample(self.B, seed=self.seed + 777, counter=counter, counter_dev=self.learn_counter,
                                  out=self.rows_buf[nxt], state=state, guard=guard, taus=self.taus_buf[nxt])
        from .fused_update import target_q
        target_q(st, rows, self.taus_buf[nxt][0], st.q_next_buf[nxt], st.na_p)

    def _learn_pipelined(self, state, guard, actor_wait):
        cur = self._parity
        nxt = 1 - cur
        if not self._primed:   # the first batch of the run (eager, before any capture)
            self._produce(cur, state, guard, 0)
            self._primed = True
        st = self.fused2
        out = ac_iqn_update_fused2(st, self.local, self.actor_opt, self.critic_opt, self.critic_grads,
                                   self.actor_grads, self.rows_buf[cur], gamma=self.gamma, sync=self.sync,
                                   actor_wait=actor_wait, taus=self.taus_buf[cur], q_next=st.q_next_buf[cur],
                                   produce=lambda: self._produce(nxt, state, guard, 1))
        self._parity = nxt
        self.learn_counter += 1
        return out

    def learn(self, state=None, guard=0, actor_wait=None):
        if self.pipeline:
            return self._learn_pipelined(state, guard, actor_wait)
        if self.per is not None:
            rows, idx = self.per.sample(self.B, seed=self.seed + 777, counter_dev=self.learn_counter,
                                        out=self.batch_rows, out_idx=self.per_idx)
            if self.fused_rb is not None:   # act() composed the online weights this iteration
                loss, gn = self.fused_rb.update(self.opt, self.grads, rows, gamma=self.gamma, n=self.n_step,
                                                sync=self.sync, seed=self.seed + 999, counter_dev=self.learn_counter,
                                                compose=False)
                self.per.update_priorities(idx, loss)
                self.learn_counter += 1
                return loss.mean(), gn
            amp = torch.autocast("cuda", dtype=self.amp_dtype) if self.amp_dtype is not None else _null()
            with amp:
                if self.rainbow_packed:
                    loss, gn = rainbow_update_rows(self.local, self.target, self.opt, self.grads, self.support,
                                                   rows, gamma=self.gamma, n=self.n_step, sync=self.sync)
                else:
                    s, a, R, ns, nt = split_rows(rows)
                    loss, gn = rainbow_update(self.local, self.target, self.opt, self.grads, self.support, s,
                                              a[:, 0].to(torch.int64), R, ns, nt, rows[:, 84], gamma=self.gamma,
                                              n=self.n_step, sync=self.sync)
            self.per.update_priorities(idx, loss)   # update_priorities(idxs, loss) (agent.py:639)
            self.learn_counter += 1
            return loss.mean(), gn
        taus = self.taus if self._fused_learner() else None   # drawn by the sampling launch
        rows = self.replay.sample(self.B, seed=self.seed + 777, counter_dev=self.learn_counter, out=self.batch_rows,
                                  state=state, guard=guard, taus=taus)
        if self.agent_type == "AC-IQN" and self.fused2 is not None:
            return ac_iqn_update_fused2(self.fused2, self.local, self.actor_opt, self.critic_opt, self.critic_grads,
                                        self.actor_grads, rows, gamma=self.gamma, sync=self.sync,
                                        actor_wait=actor_wait, taus=taus, counter=self.learn_counter)
        if self.fused_iqn is not None:
            return iqn_update_fused(self.fused_iqn, self.local, self.opt, self.grads, rows, gamma=self.gamma,
                                    sync=self.sync, act_wait=actor_wait, taus=taus[:2], counter=self.learn_counter)
        s, a, r, ns, d = split_rows(rows)
        if self.agent_type == "AC-IQN" and self.fused is not None:
            out = ac_iqn_update_fused(self.fused, self.local, self.target, self.actor_opt, self.critic_opt,
                                      self.critic_grads, self.actor_grads, s, a, r, ns, d, gamma=self.gamma,
                                      sync=self.sync, amp_dtype=self.amp_dtype)
        elif self.agent_type == "AC-IQN":
            out = ac_iqn_update(self.local, self.target, self.actor_opt, self.critic_opt, self.critic_grads,
                                self.actor_grads, s, a, r, ns, d, gamma=self.gamma, num_tau=self.num_tau,
                                sync=self.sync, amp_dtype=self.amp_dtype)
        else:
            act = a[:, 0].to(torch.int64)
            out = iqn_update(self.local, self.target, self.opt, self.grads, s, act, r, ns, d, gamma=self.gamma,
                             num_tau=self.num_tau, sync=self.sync, amp_dtype=self.amp_dtype)
        self.learn_counter += 1
        return out

    def hard_update(self):
        """soft_update with TAU = 1.0 (agent.py:643-679): target <- local."""
        with torch.no_grad():
            if self.agent_type == "AC-IQN":
                pairs = list(zip(self.target.actor.parameters(), self.local.actor.parameters())) + \
                    list(zip(self.target.critic.parameters(), self.local.critic.parameters()))
            else:
                pairs = list(zip(self.target.parameters(), self.local.parameters()))
            torch._foreach_copy_([t for t, _ in pairs], [l for _, l in pairs])
            if self.agent_type == "AC-IQN" and self.fused is not None:
                self.fused.target_pack.refresh()  # eager, outside any captured graph
            if self.agent_type == "AC-IQN" and self.fused2 is not None:
                self.fused2.target_changed()
            if self.fused_iqn is not None:
                self.fused_iqn.target_changed()
            if self.fused_rb is not None:
                self.fused_rb.target_changed()

    # ------------------------------------------------------------------ iteration
    def _iteration_body(self, do_learn):
        if not (do_learn and self.overlap and self._fused_learner()):
            self.rollout()
            out = self.learn() if do_learn else None
            self.env.advance_device()
            return out
        # the learner runs on the current stream and the rollout on a side stream: HIP graph
        # capture (ROCm 7) segfaults at capture end on a stream forked from an already forked
        # stream, and the learner forks side streams of its own (fused_update.SideStreams)
        main = torch.cuda.current_stream(self.device)
        if self._streams is None:
            self._streams = (self.roll_stream(),) + self._roll_events()
        s_roll, ev_snap, ev_act = self._streams
        # the replay state the learner samples against (after the previous iteration's push, which
        # the caller's stream joined), copied on the learner's own stream: the learner's chain then
        # starts without a cross-stream wait (each costs ~10 us in a replayed graph)
        self.ring_snap.copy_(self.replay.state)
        s_roll.wait_stream(main)
        with torch.cuda.stream(s_roll):
            self.act()
            ev_act.record(s_roll)
            env = self.env
            env.step(self.actions)
            self._push()
            env.auto_reset()
            env.advance_device()
        out = self.learn(state=self.ring_snap, guard=self.E * self.R, actor_wait=ev_act)
        main.wait_stream(s_roll)
        return out

    def iteration(self, timing=None):
        """One fused rollout+learn iteration. Returns losses (device tensors) or None."""
        do_learn = self.replay_size_host() >= self.learning_starts
        if self.graphs and do_learn and self._graph is None:
            try:
                self._capture()
            except RuntimeError as e:   # a capture the runtime refuses: keep going eagerly, loudly
                import sys
                print(f"VecTrainer: HIP graph capture failed ({e}); continuing without graphs", file=sys.stderr)
                self.graphs, self._graph = False, None
        if self.graphs and do_learn:
            if self._phase == 0:
                self._graph.replay()
            self._phase = (self._phase + 1) % self.unroll
            out = self._graph_out
        else:
            out = self._iteration_body(do_learn)
        self.env.advance_host()
        self.iterations += 1
        if do_learn:
            self.learn_steps += 1
            if self.learn_steps % self.target_update_interval == 0:
                self.hard_update()
        self.last_losses = out
        return out

    def replay_size_host(self):
        # host-side estimate avoids a device sync every iteration: exact once the buffer
        # has been observed >= learning_starts (it only grows until full)
        if getattr(self, "_replay_ready", False):
            return self.learning_starts
        n = self.per.pushed if self.per is not None else self.replay.size()
        if n >= self.learning_starts:
            self._replay_ready = True
        return n

    def roll_stream(self):
        """The rollout's stream: a dedicated one (streams.py), never an alias of the capture stream or
        of the learner's side streams."""
        return streams.stream(self.device, "roll")

    def _roll_events(self):
        return torch.cuda.Event(), torch.cuda.Event()

    def _chained(self):
        return (self.chain and self.overlap and self._fused_learner() and not self.pipeline
                and self.unroll % 2 == 0)

    def _chain_body(self):
        """self.unroll iterations with per-dependency stream ordering (captured only; see __init__)."""
        main = torch.cuda.current_stream(self.device)
        if self._streams is None:
            self._streams = (self.roll_stream(),) + self._roll_events()
        s_roll = self._streams[0]
        U = self.unroll
        ev_act = [torch.cuda.Event() for _ in range(U)]
        ev_snap = [torch.cuda.Event() for _ in range(U)]
        ev_learn = [torch.cuda.Event() for _ in range(U)]
        # the events live as long as the graph: the captured cross-stream waits may refer to them at replay
        self._chain_events = (ev_act, ev_snap, ev_learn)
        s_roll.wait_stream(main)
        out = None
        for k in range(U):
            with torch.cuda.stream(s_roll):
                if k > 0:
                    s_roll.wait_event(ev_learn[k - 1])   # the weights learn(k-1) wrote
                self.act()
                ev_act[k].record(s_roll)
                env = self.env
                env.step(self.actions)
                self._push()
                self.ring_snap2[k % 2].copy_(self.replay.state)   # what learn(k+1) samples against
                ev_snap[k].record(s_roll)
                env.auto_reset()
                env.advance_device()
            if k > 0:
                main.wait_event(ev_snap[k - 1])
            out = self.learn(state=self.ring_snap2[(k - 1) % 2], guard=self.E * self.R, actor_wait=ev_act[k])
            ev_learn[k].record(main)
        main.wait_stream(s_roll)
        return out

    def _capture(self):
        # warm up the captured region on a side stream (allocator + autograd state)
        s = streams.stream(self.device, "warmup")
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(3):
                self._iteration_body(True)
                self.env.advance_host()
        torch.cuda.current_stream(self.device).wait_stream(s)
        if self.pipeline:   # the graph's first body consumes parity 0
            while self._parity != 0:
                with torch.cuda.stream(s):
                    self._iteration_body(True)
                    self.env.advance_host()
                torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # thread_local: the RCCL process group's watchdog thread queries its work events while this
        # thread captures; under the default global mode that query invalidates the capture and the
        # watchdog aborts the process
        chained = self._chained()
        if chained:   # the ring state after the last eager push: what the graph's first learner samples against
            self.ring_snap2[(self.unroll - 1) % 2].copy_(self.replay.state)
        # captured on the dedicated capture stream: torch.cuda.graph's default is a pool stream that a
        # long process also hands out as "another" stream (streams.py)
        with torch.cuda.graph(g, stream=streams.capture_stream(self.device), capture_error_mode="thread_local"):
            if chained:
                self._graph_out = self._chain_body()
            else:
                for _ in range(self.unroll):
                    self._graph_out = self._iteration_body(True)
        self._graph = g

    def run(self, iterations):
        t0 = time.time()
        for _ in range(iterations):
            self.iteration()
        torch.cuda.synchronize(self.device)
        return time.time() - t0


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
