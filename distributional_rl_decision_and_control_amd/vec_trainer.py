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
import time

import torch

from . import streams
from .fused_update import FusedACIQNState, ac_iqn_update_fused2, learn_prologue
from .fused_iqn import FusedIQNState, iqn_update_fused
from .fused_iqn import supported as fused_iqn_supported
from .fused_rainbow import FusedRainbow
from .fused_update import supported as fused2_supported
from .learn_ops import DevicePER, DeviceReplay
from .learner import FusedAdam
from .policy.AC_IQN_model import AC_IQN_Policy
from .policy.IQN_model import IQN_Policy
from .policy.Rainbow_model import Rainbow_Policy
from .vec_env import VecMarineNavEnv

DEFAULT_NET = dict(self_dimension=7, object_dimension=5, max_object_num=5, self_feature_dimension=56,
                   object_feature_dimension=40, concat_feature_dimension=256, hidden_dimension=128)


class VecTrainer:
    def __init__(self, n_envs=4096, agent_type="AC-IQN", num_robots=5, num_obs=4, num_cores=0, min_start_goal_dis=40.0,
                 width=55.0, batch_size=4096, num_tau=32, buffer_size=4_000_000, lr=1e-4, gamma=0.99,
                 learning_starts=None, target_update_interval=2500, total_timesteps=6_000_000,
                 exploration_fraction=0.25, initial_eps=0.6, final_eps=0.05, seed=0,
                 device="cuda", sync=None, graphs=False, schedule=None, net_seed=100, overlap=True, unroll=1,
                 chain=None, operands="bf16", target_after_env=False, push_after_actor=None):
        """Every learner runs on the hand-written kernels (fused_update / fused_iqn / fused_rainbow) with
        FusedAdam; operands="f32" takes them from the f32-operand parity build (libasvrl_f32.so). Shapes
        the kernels do not take raise ValueError."""
        self.device = torch.device(device)
        self.agent_type = agent_type
        # chained schedule knob: the AC-IQN learner's target critic waits for the same iteration's env step
        # (the two then run one after the other instead of side by side; results unchanged). With the target pass
        # inside the fused critic launch (fused_update.TARGET_IN_FUSED, the default) that wait gates the whole
        # fused critic update, not only the target forward
        self.target_after_env = bool(target_after_env)
        # schedule knob: the rollout's replay push (and the reset behind it) waits for the learner's ACTOR pass
        # of the same iteration instead of running beside it (None: wherever the chained AC-IQN graph runs)
        self._paa_arg = push_after_actor
        self.push_after_actor = bool(push_after_actor)
        self.continuous = agent_type == "AC-IQN"
        self.env = VecMarineNavEnv(n_envs, num_robots, num_obs, num_cores, min_start_goal_dis, width, seed=seed,
                                   device=self.device, is_continuous=self.continuous, gamma=gamma, schedule=schedule)
        self.E, self.R = n_envs, self.env.max_robots
        self.B, self.num_tau, self.gamma = batch_size, num_tau, gamma
        self.operands = operands
        self.sync = sync
        self.seed = seed
        self.target_update_interval = target_update_interval
        self.total_timesteps = total_timesteps
        self.exploration_fraction, self.initial_eps, self.final_eps = exploration_fraction, initial_eps, final_eps
        self.learning_starts = learning_starts if learning_starts is not None else batch_size
        self.fused2 = self.fused_iqn = self.fused_rb = None
        if agent_type == "AC-IQN":
            self.local = AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1.0, 1.0], [-1.0, 1.0]],
                                       device=self.device, seed=net_seed)
            self.target = AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1.0, 1.0], [-1.0, 1.0]],
                                        device=self.device, seed=net_seed)
            for p in list(self.target.actor.parameters()) + list(self.target.critic.parameters()):
                p.requires_grad_(False)
            if not fused2_supported(self.local, batch_size, num_tau):
                raise ValueError(f"AC-IQN learner kernels: B={batch_size}, N={num_tau} (B a multiple of 32, "
                                 f"N in 8, 16, 32)")
            # clip + Adam over flat buffers (must precede the packs, which cache parameter pointers)
            self.actor_opt = FusedAdam(self.local.actor.parameters(), lr=lr, operands=operands)
            self.critic_opt = FusedAdam(self.local.critic.parameters(), lr=lr, operands=operands)
            self.actor_grads, self.critic_grads = self.actor_opt.grads, self.critic_opt.grads
            self.action_dim = 2
            self.fused2 = FusedACIQNState(self.local, self.target, batch_size, num_tau, operands, double_actor=True)
        elif agent_type == "IQN":
            self.local = IQN_Policy(**DEFAULT_NET, action_size=25, device=self.device, seed=net_seed).to(self.device)
            self.target = IQN_Policy(**DEFAULT_NET, action_size=25, device=self.device, seed=net_seed).to(self.device)
            for p in self.target.parameters():
                p.requires_grad_(False)
            if not fused_iqn_supported(self.local, batch_size, num_tau):
                raise ValueError(f"IQN learner kernels: B={batch_size}, N={num_tau}")
            self.opt = FusedAdam(self.local.parameters(), lr=lr, operands=operands)
            self.grads = self.opt.grads
            self.action_dim = 1
            self.fused_iqn = FusedIQNState(self.local, self.target, batch_size, num_tau, operands)
        elif agent_type == "Rainbow":
            # Rainbow_Policy (dueling NoisyNet C51, 51 atoms on [-1, 1]) with the prioritised n-step
            # replay in HBM, one stream per robot (agent.py:597-641, replay_memory_rainbow.py)
            self.local = Rainbow_Policy(**DEFAULT_NET, action_size=25, atoms=51, device=self.device,
                                        seed=net_seed).to(self.device)
            self.target = Rainbow_Policy(**DEFAULT_NET, action_size=25, atoms=51, device=self.device,
                                         seed=net_seed).to(self.device)
            for p in self.target.parameters():
                p.requires_grad_(False)
            self.opt = FusedAdam(self.local.parameters(), lr=lr, operands=operands)
            self.grads = self.opt.grads
            self.action_dim = 1
            self.n_step = 3
            self.support = torch.linspace(-1.0, 1.0, 51, device=self.device)
            # noisy weights, the network, loss gradient and act on hand-written kernels (fused_rainbow.py)
            self.fused_rb = FusedRainbow(self.local, self.target, batch_size, self.support, operands)
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
        self.loss_mean = torch.zeros(1, dtype=torch.float32, device=self.device)   # PER: the update's mean loss
        self.batch_rows = torch.zeros((self.B, 88), dtype=torch.float32, device=self.device)
        # the fused updates' quantile fractions (AC-IQN: target, local, actor step; IQN: the first two)
        self.taus = torch.zeros((3, self.B, self.num_tau), dtype=torch.float32, device=self.device)
        self.learn_steps = 0
        self.iterations = 0
        self.last_losses = None
        self.graphs = graphs
        self._graph = None
        # iterations per captured graph: one replay enqueues `unroll` whole iterations (the host
        # calls iteration() once per iteration; every unroll-th call replays): 10 with the chained
        # schedule at the bench shape (profiles/r02_unroll_chain_ab.txt)
        self.unroll = max(1, int(unroll))
        # observation double buffer by parity flip (no copy) unless a graph of an odd number of iterations
        # has to find the same buffers at every replay
        self.env.swap = not graphs or self.unroll % 2 == 0
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
        if self.target_after_env and not (self.fused2 is not None and self.graphs and self._chained()):
            # the knob orders two nodes of the chained AC-IQN graph; anywhere else it would be silently ignored
            # and a bench config recording it would be mislabelled
            raise ValueError("target_after_env applies only to the chained, graph-captured AC-IQN schedule")
        paa_ok = self.fused2 is not None and self.graphs and self._chained()
        if self._paa_arg is None:
            self.push_after_actor = paa_ok
        elif self.push_after_actor and not paa_ok:
            raise ValueError("push_after_actor applies only to the chained, graph-captured AC-IQN schedule")
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
        """The local policy on every robot row with the epsilon-greedy schedule on the device step counter
        (trainer.py:106-135, agent.py:207-250,308-324), one kernel per agent type."""
        args = (self.env.obs_cur, self.actions, self.env.counter, self.E, self.total_timesteps,
                self.exploration_fraction, self.initial_eps, self.final_eps, self.seed + 4242)
        if self.fused_rb is not None:   # composed noisy weights, logits, head: expected Q, argmax, explore
            self.fused_rb.act(*args)
        elif self.fused_iqn is not None:   # K = 32 quantiles per robot, mean, argmax, explore
            self.fused_iqn.act(*args)
        else:   # actor on every robot row, explore
            self.fused2.act(*args)

    def _push(self, snap=None):
        """The replay push of every robot that acted; for the uniform ring it is one launch that also
        increments the env step counter (and writes the new ring state to `snap` when given). Returns
        whether the counter was incremented."""
        env = self.env
        if self.per is not None:   # ReplayMemory.append of every robot that acted (trainer.py:163-164), and the
            # step counter advanced in the push's last launch
            self.per.push(env.obs_cur, env.cnt_next, self.actions[:, :1], env.batch.reward, env.batch.done,
                          step_counter=env.counter)
            return True
        self.replay.push(env.obs_cur, env.obs_next, env.cnt_next, self.actions[:, :self.action_dim],
                         env.batch.reward, env.batch.done, snap=snap, counter_inc=env.counter)
        return True

    def rollout(self, snap=None):
        """act, env step, replay push, device reset and the step counter (trainer.py:142-172)."""
        self.act()
        self.env.step(self.actions)
        counted = self._push(snap)
        self.env.auto_reset(counted)
        self.env.advance_device(counted)

    def learn(self, state=None, guard=0, actor_wait=None, target_wait=None, actor_done=None):
        """One learn step of batch B: sample (uniform ring, or the prioritised tree for Rainbow) and the
        agent's fused update. state / guard: the ring snapshot to sample against and the newest entries to
        skip (the overlapped schedule); actor_wait: an event to wait for before the actor's weights change."""
        if self.per is not None:
            rows, idx = self.per.sample(self.B, seed=self.seed + 777, counter_dev=self.learn_counter,
                                        out=self.batch_rows, out_idx=self.per_idx)
            # act() composed the online noisy weights this iteration
            loss, gn = self.fused_rb.update(self.opt, self.grads, rows, gamma=self.gamma, n=self.n_step,
                                            sync=self.sync, seed=self.seed + 999, counter_dev=self.learn_counter,
                                            compose=False)
            # update_priorities(idxs, loss) (agent.py:639); the reported loss mean and the learn counter in its last
            # launch
            self.per.update_priorities(idx, loss, mean_out=self.loss_mean, learn_counter=self.learn_counter)
            return self.loss_mean[0], gn
        if self.fused2 is not None:
            # one launch: the draw (rows + the update's quantile fractions), the actor's training forward
            # and the target actor
            rows = learn_prologue(self.fused2, self.replay, self.taus, self.seed + 777, counter_dev=self.learn_counter,
                                  out=self.batch_rows, state=state, guard=guard)
            return ac_iqn_update_fused2(self.fused2, self.local, self.actor_opt, self.critic_opt, self.critic_grads,
                                        self.actor_grads, rows, gamma=self.gamma, sync=self.sync,
                                        actor_wait=actor_wait, taus=self.taus, counter=self.learn_counter,
                                        prologue_done=True, target_wait=target_wait, actor_done=actor_done)
        # the update's quantile fractions are drawn by the sampling launch
        rows = self.replay.sample(self.B, seed=self.seed + 777, counter_dev=self.learn_counter, out=self.batch_rows,
                                  state=state, guard=guard, taus=self.taus)
        return iqn_update_fused(self.fused_iqn, self.local, self.opt, self.grads, rows, gamma=self.gamma,
                                sync=self.sync, act_wait=actor_wait, taus=self.taus[:2], counter=self.learn_counter)

    def hard_update(self):
        """soft_update with TAU = 1.0 (agent.py:643-679): target <- local."""
        with torch.no_grad():
            if self.agent_type == "AC-IQN":
                pairs = list(zip(self.target.actor.parameters(), self.local.actor.parameters())) + \
                    list(zip(self.target.critic.parameters(), self.local.critic.parameters()))
            else:
                pairs = list(zip(self.target.parameters(), self.local.parameters()))
            torch._foreach_copy_([t for t, _ in pairs], [l for _, l in pairs])
            if self.fused2 is not None:   # eager, outside any captured graph
                self.fused2.target_changed()
            if self.fused_iqn is not None:
                self.fused_iqn.target_changed()
            if self.fused_rb is not None:
                self.fused_rb.target_changed()

    @torch.no_grad()
    def load_policies(self, local, target):
        """Start from the given networks (a drop-in Agent's policy_local / policy_target, e.g. after its
        load_model): their weights are copied in place into this trainer's networks (whose parameters
        are views of the optimisers' flat buffers) and every weight image is re-packed. Eager, before
        the first captured graph."""
        assert self._graph is None, "load_policies before the first captured iteration"
        pairs = [(self.local, local), (self.target, target)]
        for dst, src in pairs:
            mods = [(dst.actor, src.actor), (dst.critic, src.critic)] if hasattr(dst, "actor") else [(dst, src)]
            for d, s in mods:
                sd = s.state_dict()
                for name, t in d.state_dict(keep_vars=True).items():
                    t.data.copy_(sd[name].to(device=t.device, dtype=t.dtype))
        if self.fused2 is not None:
            self.fused2.local_trunk.refresh()
            self.fused2.actor.refresh()
            self.fused2.target_changed()
        if self.fused_iqn is not None:
            self.fused_iqn.local.refresh()
            self.fused_iqn.target_changed()
        if self.fused_rb is not None:
            self.fused_rb.pack.compose()
            self.fused_rb.img.refresh()
            self.fused_rb.target_changed()

    # ------------------------------------------------------------------ iteration
    def _iteration_body(self, do_learn):
        if not (do_learn and self.overlap and self.per is None):
            # the learner samples after the push: only the act -> push order of rollout() matters
            self.rollout()
            return self.learn() if do_learn else None
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
            counted = self._push()
            env.auto_reset(counted)
            env.advance_device(counted)
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
        return self.chain and self.overlap and self.per is None and self.unroll % 2 == 0

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
        ev_env = [torch.cuda.Event() for _ in range(U)]
        ev_actor = [torch.cuda.Event() for _ in range(U)]
        # the events live as long as the graph: the captured cross-stream waits may refer to them at replay
        self._chain_events = (ev_act, ev_snap, ev_learn, ev_env, ev_actor)
        tae = self.target_after_env and self.fused2 is not None
        paa = self.push_after_actor and self.fused2 is not None
        s_roll.wait_stream(main)
        out = None

        def push_reset(k):
            self._push(snap=self.ring_snap2[k % 2])   # + the ring state learn(k+1) samples against
            ev_snap[k].record(s_roll)
            self.env.auto_reset(True)
            self.env.advance_device(True)

        for k in range(U):
            with torch.cuda.stream(s_roll):
                if k > 0:
                    s_roll.wait_event(ev_learn[k - 1])   # the weights learn(k-1) wrote
                self.act()
                ev_act[k].record(s_roll)
                self.env.step(self.actions)
                if tae:
                    ev_env[k].record(s_roll)
                if not paa:
                    push_reset(k)
            if k > 0:
                main.wait_event(ev_snap[k - 1])
            out = self.learn(state=self.ring_snap2[(k - 1) % 2], guard=self.E * self.R, actor_wait=ev_act[k],
                             target_wait=ev_env[k] if tae else None, actor_done=ev_actor[k] if paa else None)
            ev_learn[k].record(main)
            if paa:
                with torch.cuda.stream(s_roll):
                    s_roll.wait_event(ev_actor[k])
                    push_reset(k)
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
