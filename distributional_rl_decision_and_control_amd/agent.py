"""Agent -- drop-in for rfarl.agent.Agent (agent.py:18-707) for the distributional agents.

Same constructor (keyword names and defaults), fields (agent_type, GAMMA, BATCH_SIZE,
training, memory, policy_local/policy_target), act_* / train / soft_update /
save_latest_model / load_model surfaces and return types. Differences:
  * tensors live on the GPU: `device="cpu"` (the reference default) selects the current
    HIP device -- the kernels have no CPU implementation and no CPU fallback;
  * train_AC_IQN / train_IQN run the hand-written learner of the batched trainer
    (fused_update.ac_iqn_update_fused2, fused_iqn.iqn_update_fused) built with f32 operands
    (libasvrl_f32.so: the reference's fp32 arithmetic, pinned to its train_* outputs at 1e-5 by
    tests/test_learner_golden_gpu.py and test_agent_gpu.py); set_learner("fused-bf16") selects the
    bf16-operand training build, set_learner("torch") the torch-autograd restatement with the HIP
    quantile-Huber kernel (learner.py). train_Rainbow runs the hand-written Rainbow learner
    (fused_rainbow.FusedRainbow: network, C51 projection, loss, backward and weight-gradient kernels)
    of the same operand build, pinned to the reference's train_Rainbow by
    tests/test_rainbow_golden_gpu.py; set_learner("torch") (or network dims the kernels do not take)
    runs learner.rainbow_update (torch autograd + the C51 kernel). Every learner's optimiser: FusedAdam
    (asvrl_adam_*, pinned to torch.optim.Adam at 1e-5) for AC-IQN / IQN, torch.optim.Adam for Rainbow
    and DQN;
  * load_model rebuilds the optimizers for the loaded networks (the reference keeps
    optimizing the replaced ones, agent.py:684-698 vs :75-76,98);
  * DQN runs as the reference's plain torch update (BASELINE config 1 is the DQN plumbing run of
    train_RL_agents.py); DDPG / SAC (non-distributional baselines) are out of scope and raise.
"""
import copy
import random
import warnings

import numpy as np
import torch
import torch.nn.functional as F

from . import _abi
from . import fused_iqn, fused_rainbow, fused_update
from .learn_ops import rows_from_batch
from .learner import FlatGrads, FusedAdam, ac_iqn_update, iqn_update, rainbow_update
from .policy.AC_IQN_model import AC_IQN_Policy
from .policy.DQN_model import DQN_Policy
from .policy.IQN_model import IQN_Policy
from .policy.Rainbow_model import Rainbow_Policy
from .policy.replay_memory_rainbow import ReplayMemory
from .utils.replay_buffer import ReplayBuffer

DISTRIBUTIONAL = ("AC-IQN", "IQN", "Rainbow")
SUPPORTED = DISTRIBUTIONAL + ("DQN",)
# learners of train_AC_IQN / train_IQN: the hand-written kernels with f32 operands (default, the
# reference's arithmetic), the same kernels with bf16 operands (the batched trainer's build), or
# the torch-autograd restatement
LEARNERS = {"fused-f32": "f32", "fused-bf16": "bf16", "torch": None}


def resolve_device(device):
    """The reference passes device strings like "cpu" (train_RL_agents.py -D); the hot path
    needs the GPU, so "cpu"/None map to the current HIP device. No device -> error."""
    _abi.lib()
    if not torch.cuda.is_available():
        raise _abi.AsvrlError("the rfarl hot path runs on an MI355X (HIP) device; none is visible")
    if device is None or str(device) == "cpu":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


def _mode_dependent(module):
    """True when train() / eval() changes what `module` computes (dropout or batch-norm layers); cached on the
    module (its layers do not change after construction)."""
    v = getattr(module, "_asvrl_mode_dependent", None)
    if v is None:
        kinds = (torch.nn.modules.dropout._DropoutNd, torch.nn.modules.batchnorm._BatchNorm)
        v = any(isinstance(m, kinds) for m in module.modules())
        object.__setattr__(module, "_asvrl_mode_dependent", v)
    return v


class Agent:
    def __init__(self, self_dimension=7, object_dimension=5, max_object_num=5, self_feature_dimension=56,
                 object_feature_dimension=40, concat_feature_dimension=256, hidden_dimension=128,
                 value_ranges_of_action=[[-1.0, 1.0], [-1.0, 1.0]], action_size=25, multi_steps=3, BATCH_SIZE=64,
                 BUFFER_SIZE=1_000_000, LR=1e-4, TAU=1.0, GAMMA=0.99, device="cpu", seed=0, training=True,
                 agent_type=None):
        self.device = resolve_device(device)
        self.LR = LR
        self.TAU = TAU
        self.GAMMA = GAMMA
        self.BUFFER_SIZE = BUFFER_SIZE
        self.BATCH_SIZE = BATCH_SIZE
        self.training = training
        self.value_ranges_of_action = copy.deepcopy(value_ranges_of_action)
        self.action_size = action_size
        self.agent_type = agent_type
        self._rb_seed = int(seed) + 999   # the kernel path's target-noise Philox stream
        self.num_tau = 8  # training quantiles N = N' (AC_IQN_model.py:462, IQN_model.py:74)
        self.tau_override = None  # optional list of pre-drawn taus for the next train() (tests)
        self.learner = "fused-f32"
        self._fused = None   # (B, N) -> FusedACIQNState / FusedIQNState, built on the first train()
        self._net_args = (self_dimension, object_dimension, max_object_num, self_feature_dimension,
                          object_feature_dimension, concat_feature_dimension, hidden_dimension)
        if agent_type not in SUPPORTED:
            if agent_type in ("DDPG", "SAC"):
                raise NotImplementedError(f"{agent_type} is a non-distributional baseline, outside this "
                                          "framework's hot path (SURVEY.md section 2, row 14)")
            raise RuntimeError("Agent type not implemented!")
        if training:
            self.policy_local = self._make_policy(seed, value_ranges_of_action, action_size)
            self.policy_target = self._make_policy(seed, value_ranges_of_action, action_size)
            self._make_optimizers()
            if agent_type == "Rainbow":
                self.atoms = 51
                self.Vmin = -1.0
                self.Vmax = 1.0
                self.support = torch.linspace(self.Vmin, self.Vmax, self.atoms).to(self.device)
                self.delta_z = (self.Vmax - self.Vmin) / (self.atoms - 1)
                self.n = multi_steps
                self.memory = ReplayMemory(self.device, BUFFER_SIZE)
            else:
                self.memory = ReplayBuffer(BUFFER_SIZE, BATCH_SIZE, object_dimension, max_object_num,
                                           device=self.device)

    # ------------------------------------------------------------------ construction
    def _make_policy(self, seed, value_ranges_of_action, action_size):
        a = self._net_args
        if self.agent_type == "AC-IQN":
            return AC_IQN_Policy(*a, value_ranges_of_action, self.device, seed)
        if self.agent_type == "IQN":
            return IQN_Policy(*a, action_size, self.device, seed).to(self.device)
        if self.agent_type == "DQN":
            return DQN_Policy(*a, action_size, self.device, seed).to(self.device)
        return Rainbow_Policy(*a, action_size, 51, self.device, seed).to(self.device)

    def _make_optimizers(self):
        """optim.Adam(lr) + clip 0.5 (agent.py:75-76,98): FusedAdam (asvrl_adam_*) of the learner's
        operand build for AC-IQN / IQN, torch Adam for Rainbow / DQN."""
        self._fused = None
        ops = LEARNERS[self.learner] or "bf16"
        if self.agent_type == "AC-IQN":
            self.actor_optimizer = FusedAdam(self.policy_local.actor.parameters(), lr=self.LR, operands=ops)
            self.critic_optimizer = FusedAdam(self.policy_local.critic.parameters(), lr=self.LR, operands=ops)
            self.actor_grads, self.critic_grads = self.actor_optimizer.grads, self.critic_optimizer.grads
        elif self.agent_type == "IQN":
            self.optimizer = FusedAdam(self.policy_local.parameters(), lr=self.LR, operands=ops)
            self.grads = self.optimizer.grads
        else:
            self.grads = FlatGrads(self.policy_local.parameters())
            self.optimizer = torch.optim.Adam(self.policy_local.parameters(), lr=self.LR)

    def set_learner(self, learner):
        """Select train_AC_IQN / train_IQN's learner (LEARNERS); rebuilds the optimisers (fresh Adam
        state, as load_model does)."""
        if learner not in LEARNERS:
            raise ValueError(f"learner must be one of {sorted(LEARNERS)}")
        self.learner = learner
        if self.training:
            self._make_optimizers()

    def _fused_state(self, B):
        """The fused update's packs and buffers for batch B and N = self.num_tau, or None when the
        torch learner is selected or the network shape is not the kernels' (supported())."""
        ops = LEARNERS[self.learner]
        if ops is None:
            return None
        key = (B, self.num_tau)
        if self._fused is None or self._fused[0] != key:
            if self.agent_type == "Rainbow":
                ok = fused_rainbow.supported(self.policy_local, B)
                st = fused_rainbow.FusedRainbow(self.policy_local, self.policy_target, B, self.support,
                                                operands=ops) if ok else None
            elif self.agent_type == "AC-IQN":
                ok = fused_update.supported(self.policy_local, B, self.num_tau)
                st = fused_update.FusedACIQNState(self.policy_local, self.policy_target, B, self.num_tau,
                                                  operands=ops) if ok else None
            else:
                ok = fused_iqn.supported(self.policy_local, B, self.num_tau)
                # nothing runs beside the drop-in's update: the target's max inside the fused launch (bf16 build)
                st = fused_iqn.FusedIQNState(self.policy_local, self.policy_target, B, self.num_tau,
                                             operands=ops, target_in_fused=True) if ok else None
            if st is None:
                # not silent: this batch / network shape runs on the torch-autograd learner (learner.py), not on
                # the hand-written kernels
                warnings.warn(f"Agent({self.agent_type}): batch {B}, num_tau {self.num_tau} or the network shape is "
                              "not one the fused kernels take; this learn step runs the torch-autograd learner",
                              RuntimeWarning, stacklevel=3)
            self._fused = (key, st)
        return self._fused[1]

    # ------------------------------------------------------------------ acting (agent.py:207-324)
    def state_to_tensor(self, states):
        self_state_batch, object_batch, object_batch_mask = states
        self_t = torch.tensor(self_state_batch).float().to(self.device)
        if len(object_batch) == 0:
            return self_t, None, None
        return (self_t, torch.tensor(object_batch).float().to(self.device),
                torch.tensor(object_batch_mask).float().to(self.device))

    def _batch1(self, state):
        return self.state_to_tensor(self.memory.state_batch([state]))

    def act_ac_iqn(self, state, eps=0.0, cvar=1.0, use_eval=True):
        if random.random() > eps:
            s = self._batch1(state)
            self.policy_local.actor.eval() if use_eval else self.policy_local.actor.train()
            with torch.no_grad():
                action = self.policy_local.actor(s).cpu().data.numpy()[0].tolist()
            self.policy_local.actor.train()
        else:
            action = [np.random.uniform(low=lo, high=hi) for lo, hi in self.value_ranges_of_action]
        return action

    def act_ac_iqn_robots(self, states, eps=0.0, use_eval=True):
        """act_ac_iqn for several robots' states in one actor call: each robot in order draws its
        random.random() and, exploring, its np.random.uniform actions exactly as the per-robot calls would; the
        greedy robots' actions come from ONE batched forward (equal to the batch-1 forwards up to the GEMM's
        summation order). The drop-in Trainer's per-step acts (trainer.py:138-151 calls act per robot)."""
        actions, greedy = [None] * len(states), []
        for i in range(len(states)):
            if random.random() > eps:
                greedy.append(i)
            else:
                actions[i] = [np.random.uniform(low=lo, high=hi) for lo, hi in self.value_ranges_of_action]
        if greedy:
            s = self.state_to_tensor(self.memory.state_batch([states[i] for i in greedy]))
            net = self.policy_local.actor
            # the eval / train switch is a no-op for a network without mode-dependent layers (the Actor has none):
            # skipped there (a recursive module walk per call, ~80 us per step of the drop-in loop)
            toggle = _mode_dependent(net)
            if toggle:
                net.eval() if use_eval else net.train()
            with torch.no_grad():
                a = net(s).cpu().data.numpy()
            if toggle:
                net.train()
            for k, i in enumerate(greedy):
                actions[i] = a[k].tolist()
        return actions

    def act_iqn(self, state, eps=0.0, cvar=1.0, use_eval=True, taus=None):
        s = self._batch1(state)
        self.policy_local.eval() if use_eval else self.policy_local.train()
        with torch.no_grad():
            quantiles, taus = self.policy_local(s, self.policy_local.K, cvar, taus=taus)
            action_values = quantiles.mean(dim=1)
        self.policy_local.train()
        if random.random() > eps:
            action = np.argmax(action_values.cpu().data.numpy())
        else:
            action = random.choice(np.arange(self.action_size))
        return action, quantiles.cpu().data.numpy(), taus.cpu().data.numpy()

    def act_rainbow(self, state, eps=0.0, use_eval=True):
        s = self._batch1(state)
        self.policy_local.eval() if use_eval else self.policy_local.train()
        with torch.no_grad():
            p = self.policy_local(s)
        self.policy_local.train()
        if random.random() > eps:
            return (p * self.support).sum(2).argmax(1).item()
        return random.choice(np.arange(self.action_size))

    def act_dqn(self, state, eps=0.0, use_eval=True):  # agent.py:271-287
        s = self._batch1(state)
        self.policy_local.eval() if use_eval else self.policy_local.train()
        with torch.no_grad():
            action_values = self.policy_local(s)
        self.policy_local.train()
        if random.random() > eps:
            return np.argmax(action_values.cpu().data.numpy())
        return random.choice(np.arange(self.action_size))

    def act_ddpg(self, *a, **k):
        raise NotImplementedError("DDPG is outside this framework's hot path")

    act_sac = act_ddpg

    # ------------------------------------------------------------------ learning (agent.py:370-641)
    def train(self):
        if self.agent_type == "AC-IQN":
            return self.train_AC_IQN()
        if self.agent_type == "IQN":
            return self.train_IQN()
        if self.agent_type == "Rainbow":
            return self.train_Rainbow()
        if self.agent_type == "DQN":
            return self.train_DQN()
        raise RuntimeError("Agent type not implemented!")

    def _taus(self, k):
        t, self.tau_override = self.tau_override, None
        if t is None:
            return (None,) * k
        return tuple(torch.as_tensor(x, device=self.device, dtype=torch.float32) for x in t)

    def _fused_taus(self, k, B):
        t = self._taus(k)
        if t[0] is None:
            return None
        return torch.stack([x.reshape(B, self.num_tau) for x in t]).contiguous()

    def train_AC_IQN(self):
        s, a, r, ns, d = self.memory.sample()
        st = self._fused_state(s[0].shape[0])
        if st is not None:   # the hand-written learner (agent.py:386-432)
            B = s[0].shape[0]
            cl, al, _, _ = fused_update.ac_iqn_update_fused2(
                st, self.policy_local, self.actor_optimizer, self.critic_optimizer, self.critic_grads,
                self.actor_grads, rows_from_batch(s, a, r, ns, d), gamma=self.GAMMA, taus=self._fused_taus(3, B))
            return cl.cpu().numpy(), al.cpu().numpy()
        cl, al, _, _ = ac_iqn_update(self.policy_local, self.policy_target, self.actor_optimizer,
                                     self.critic_optimizer, self.critic_grads, self.actor_grads, s, a, r, ns, d,
                                     gamma=self.GAMMA, num_tau=self.num_tau, taus=self._taus(3))
        return cl.cpu().numpy(), al.cpu().numpy()

    def train_IQN(self):
        s, a, r, ns, d = self.memory.sample()
        st = self._fused_state(s[0].shape[0])
        if st is not None:   # the hand-written learner (agent.py:434-476)
            B = s[0].shape[0]
            loss, _ = fused_iqn.iqn_update_fused(st, self.policy_local, self.optimizer, self.grads,
                                                 rows_from_batch(s, a[:, :1], r, ns, d), gamma=self.GAMMA,
                                                 taus=self._fused_taus(2, B))
            return loss.cpu().numpy()
        loss, _ = iqn_update(self.policy_local, self.policy_target, self.optimizer, self.grads, s,
                             a[:, 0].to(torch.int64), r, ns, d, gamma=self.GAMMA, num_tau=self.num_tau,
                             taus=self._taus(2))
        return loss.cpu().numpy()

    def train_Rainbow(self, reset_target_noise=True):
        """agent.py:597-641. reset_target_noise=False keeps the target's noise buffers (the parity tests
        inject the reference's draw); otherwise reset_noise() draws them (Philox in the kernel path)."""
        idxs, s, a, R, ns, nt, w = self.memory.sample(self.BATCH_SIZE)
        st = self._fused_state(s[0].shape[0])
        if st is not None:   # the hand-written learner
            rows = rows_from_batch(s, a.reshape(-1, 1).float(), R, ns, nt)
            rows[:, 84] = w.reshape(-1)
            self._rb_step = getattr(self, "_rb_step", 0) + 1
            ctr = torch.full((1,), self._rb_step, dtype=torch.int64, device=self.device)
            loss, _ = st.update(self.optimizer, self.grads, rows, gamma=self.GAMMA, n=self.n, vmin=self.Vmin,
                                vmax=self.Vmax, seed=self._rb_seed, counter_dev=ctr,
                                reset_target=reset_target_noise)
        else:
            loss, _ = rainbow_update(self.policy_local, self.policy_target, self.optimizer, self.grads, self.support,
                                     s, a, R, ns, nt, w, gamma=self.GAMMA, n=self.n, vmin=self.Vmin, vmax=self.Vmax,
                                     reset_target_noise=reset_target_noise)
        loss = loss.cpu().numpy().copy()
        self.memory.update_priorities(idxs, loss)
        return loss

    def train_DQN(self):
        """agent.py:518-545: max-over-actions target, smooth L1, clip 0.5, Adam (plain torch)."""
        s, a, r, ns, d = self.memory.sample()
        actions = a[:, :1].to(torch.int64)
        self.optimizer.zero_grad()
        with torch.no_grad():
            q_next = self.policy_target(ns).max(dim=1, keepdim=True)[0]
            q_targets = r + (1 - d) * self.GAMMA * q_next
        q_expected = self.policy_local(s).gather(1, actions)
        loss = F.smooth_l1_loss(q_expected, q_targets)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.policy_local.parameters(), 0.5)
        self.optimizer.step()
        return loss.detach().cpu().numpy()

    def soft_update(self):
        """theta_t <- TAU theta + (1 - TAU) theta_t (agent.py:643-679)."""
        if self.agent_type == "AC-IQN":
            pairs = list(zip(self.policy_target.actor.parameters(), self.policy_local.actor.parameters())) + \
                list(zip(self.policy_target.critic.parameters(), self.policy_local.critic.parameters()))
        else:
            pairs = list(zip(self.policy_target.parameters(), self.policy_local.parameters()))
        with torch.no_grad():
            for t, l in pairs:
                t.data.copy_(self.TAU * l.data + (1.0 - self.TAU) * t.data)
        if self._fused is not None and self._fused[1] is not None:
            self._fused[1].target_changed()   # re-pack the target networks' weight images

    def save_latest_model(self, directory):
        self.policy_local.save(directory)

    def load_model(self, path, device="cpu"):
        dev = resolve_device(device)
        cls = {"AC-IQN": AC_IQN_Policy, "IQN": IQN_Policy, "Rainbow": Rainbow_Policy,
               "DQN": DQN_Policy}[self.agent_type]
        self.policy_local = cls.load(path, dev)
        if self.training:
            self._make_optimizers()
