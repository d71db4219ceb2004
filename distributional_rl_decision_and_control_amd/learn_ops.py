"""Learner operators on the gfx950 kernels: quantile-Huber loss, C51 projection, replay ring.

All three run only through libasvrl.so (no torch fallback for the ops themselves).
"""
import ctypes as C

import torch

from . import _abi
from ._abi import OBS_DIM, TR_DIM


# ---------------------------------------------------------------------- quantile Huber
class _QuantileHuber(torch.autograd.Function):
    """Forward = agent.py:406-412 quantile-Huber loss (mean over batch, mean over target
    quantiles, sum over expected quantiles); backward = d/d qe from the same kernel."""

    @staticmethod
    def forward(ctx, qt, qe, tau, kappa):
        qt = qt.detach().float().contiguous()
        qe_c = qe.detach().float().contiguous()
        tau = tau.detach().float().contiguous()
        B, N = qe_c.shape
        Np = qt.shape[1]
        assert qt.shape[0] == B and tau.shape == (B, N)
        row = torch.empty(B, dtype=torch.float32, device=qe.device)
        loss = torch.empty((), dtype=torch.float32, device=qe.device)
        dqe = torch.empty_like(qe_c)
        rc = _abi.lib().asvrl_quantile_huber(_abi.ptr(qt), _abi.ptr(qe_c), _abi.ptr(tau), B, N, Np, float(kappa), 1.0,
                                             _abi.ptr(row), _abi.ptr(loss), _abi.ptr(dqe), _abi.stream_ptr())
        _abi.check(rc, "asvrl_quantile_huber")
        ctx.save_for_backward(dqe)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dqe,) = ctx.saved_tensors
        return None, dqe * g, None, None


def quantile_huber_loss(q_targets, q_expected, taus, kappa=1.0):
    """q_targets (B, N') detached targets, q_expected (B, N), taus (B, N) or (B, N, 1)."""
    if taus.dim() == 3:
        taus = taus.squeeze(-1)
    return _QuantileHuber.apply(q_targets, q_expected, taus, kappa)


# ---------------------------------------------------------------------- C51
def c51_project(pns_a, returns, nonterminal, support, vmin=-1.0, vmax=1.0, gamma_n=0.99 ** 3, out=None):
    """Target distribution m of agent.py:616-631 (bit-identical to the reference's CPU f32).

    gamma_n and delta_z are rounded to f32 as torch does for python scalars against f32
    tensors; nonterminal may be (B,) or (B, 1)."""
    pns_a = pns_a.float().contiguous()
    B, atoms = pns_a.shape

    def col(t):   # a strided f32 column (e.g. of the replay rows) is read in place, anything else copied
        t = t.float()
        if t.dim() == 2 and t.shape[1] == 1:
            t = t[:, 0]
        if t.dim() != 1 or t.shape[0] != B or t.stride(0) < 1:
            t = t.reshape(B).contiguous()
        return t
    R, nt = col(returns), col(nonterminal)
    sup = support.float().contiguous()
    m = out if out is not None else torch.empty_like(pns_a)
    dz = float(torch.tensor((vmax - vmin) / (atoms - 1), dtype=torch.float32))
    g32 = float(torch.tensor(gamma_n, dtype=torch.float32))
    rc = _abi.lib().asvrl_c51_project_ex(_abi.ptr(pns_a), _abi.ptr(R), R.stride(0), _abi.ptr(nt), nt.stride(0),
                                         _abi.ptr(sup), B, atoms, float(vmin), float(vmax), dz, g32, _abi.ptr(m),
                                         _abi.stream_ptr())
    _abi.check(rc, "asvrl_c51_project")
    return m


# ---------------------------------------------------------------------- replay ring
class DeviceReplay:
    """HBM-resident ring of transitions (ReplayBuffer, replay_buffer.py:6-69).

    Row layout (f32, ASVRL_TR_DIM = 88): obs 40 | next obs 40 | action 2 | reward | done | pad.
    obs rows are the packed state_batch layout: self 7 | objects 5x5 | mask 5 | pad 3.
    head/size live in device memory so push/sample can be captured in a HIP graph."""

    def __init__(self, capacity, device="cuda"):
        _abi.lib()
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.ring = torch.zeros((self.capacity, TR_DIM), dtype=torch.float32, device=self.device)
        self.state = torch.zeros(2, dtype=torch.int64, device=self.device)  # head, size
        self._work = None
        self._n_host = 0  # host mirror for the compat path (exact when fed by add())

    def push(self, obs_prev, obs_next, obj_cnt_next, actions, reward, done, stream=None, snap=None,
             counter_inc=None):
        """ReplayBuffer.add of every row whose obj_cnt_next >= 0, in row order, in one launch. actions:
        [n, >= 1] f64 rows (the first 1 or 2 columns are stored, any row stride); snap: an int64[2] that
        receives the new {head, size}; counter_inc: an int64 device counter incremented by the launch."""
        n = obs_prev.shape[0]
        if self._work is None or self._work.numel() < (n + 255) // 256 + 1:
            self._work = torch.zeros((n + 255) // 256 + 1, dtype=torch.int32, device=self.device)
        if actions.dim() == 1:
            adim, ald = 1, 1
        else:
            assert actions.stride(1) == 1, "action rows must be contiguous"
            adim, ald = min(actions.shape[1], 2), actions.stride(0)
        assert actions.dtype == torch.float64 and reward.dtype == torch.float64
        rc = _abi.lib().asvrl_replay_push_ex(_abi.ptr(obs_prev), _abi.ptr(obs_next), _abi.ptr(obj_cnt_next),
                                             _abi.ptr(actions), adim, ald, _abi.ptr(reward), _abi.ptr(done), n,
                                             _abi.ptr(self.ring), self.capacity, _abi.ptr(self.state),
                                             _abi.ptr(self._work), _abi.ptr(snap), _abi.ptr(counter_inc),
                                             _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_replay_push")

    def write_rows(self, rows, slots, stream=None):
        rc = _abi.lib().asvrl_replay_write_rows(_abi.ptr(rows), _abi.ptr(slots), rows.shape[0], _abi.ptr(self.ring),
                                                _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_replay_write_rows")

    def size(self):
        return int(self.state[1].item())

    def gather(self, indices, out=None, stream=None):
        """Rows at deque positions `indices` (0 = oldest), device int64."""
        B = indices.shape[0]
        out = out if out is not None else torch.empty((B, TR_DIM), dtype=torch.float32, device=self.device)
        rc = _abi.lib().asvrl_replay_sample(_abi.ptr(self.ring), self.capacity, _abi.ptr(self.state),
                                            _abi.ptr(indices), B, 0, 0, None, 0, _abi.ptr(out), None, None, 0, 0,
                                            _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_replay_sample")
        return out

    def sample(self, B, seed=0, counter=0, counter_dev=None, out=None, stream=None, state=None, guard=0, taus=None):
        """B rows drawn uniformly with replacement on the device (Philox). `state`: a {head, size}
        snapshot to sample against (default: the live ring state); `guard`: skip the oldest
        entries a concurrent push of up to `guard` rows may overwrite. taus: optional (sets, B, N)
        f32 buffer filled with U[0, 1) quantile fractions by the same launch."""
        out = out if out is not None else torch.empty((B, TR_DIM), dtype=torch.float32, device=self.device)
        st = state if state is not None else self.state
        ts, tn = (taus.shape[0], taus.shape[2]) if taus is not None else (0, 0)
        if taus is not None:
            assert taus.is_contiguous() and taus.shape[1] == B and taus.dtype == torch.float32
        rc = _abi.lib().asvrl_replay_sample(_abi.ptr(self.ring), self.capacity, _abi.ptr(st), None, B,
                                            int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF,
                                            _abi.ptr(counter_dev), int(guard), _abi.ptr(out), None, _abi.ptr(taus),
                                            ts, tn, _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_replay_sample")
        return out


def split_rows(rows):
    """(B, 88) replay rows -> (states, actions, rewards, next_states, dones) in the shapes
    Agent.train_* builds (agent.py:387-392): states = (self (B,7), objs (B,5,5), mask (B,5))."""
    B = rows.shape[0]
    s = (rows[:, 0:7], rows[:, 7:32].reshape(B, 5, 5), rows[:, 32:37])
    ns = (rows[:, OBS_DIM:OBS_DIM + 7], rows[:, OBS_DIM + 7:OBS_DIM + 32].reshape(B, 5, 5),
          rows[:, OBS_DIM + 32:OBS_DIM + 37])
    return s, rows[:, 80:82], rows[:, 82:83], ns, rows[:, 83:84]


def rows_from_batch(states, actions, rewards, next_states, dones):
    """The inverse of split_rows: (B, 88) f32 replay rows from Agent.train_*'s batch tensors (objects /
    mask may be None: state_batch's all-empty case, numerically all-masked, AC_IQN_model.py:293-294);
    actions (B, 1) or (B, 2)."""
    B = states[0].shape[0]
    rows = torch.zeros(B, 88, dtype=torch.float32, device=states[0].device)
    for c, st in ((0, states), (OBS_DIM, next_states)):
        rows[:, c:c + 7] = st[0]
        if st[1] is not None:
            rows[:, c + 7:c + 32] = st[1].reshape(B, 25)
            rows[:, c + 32:c + 37] = st[2]
    a = actions.reshape(B, -1)
    rows[:, 80:80 + a.shape[1]] = a
    rows[:, 82] = rewards.reshape(B)
    rows[:, 83] = dones.reshape(B)
    return rows


# ---------------------------------------------------------------------- prioritised replay
class DevicePER:
    """Rainbow's prioritised n-step replay (ReplayMemory + SegmentTree,
    replay_memory_rainbow.py:14-196) resident in HBM (asvrl_per_*).

    `stride` slots per time step: stride = 1 is the reference's single append sequence (its
    n-step window spans whatever was appended next); stride = E*R gives every robot of the
    batch its own stream, so each window is one robot's trajectory. Capacity is rounded down to
    a multiple of stride; the sum tree has next_pow2(capacity) leaves (<= 2^22). deferred=True
    (the batched trainer): a slot's priority enters the tree only once the push n steps later
    completes its window, so sampling never meets the reference's rejection case.

    sample() returns (rows [B, 88], tree_idx [B]): obs 0:40 | n-th next obs 40:80 | action 80 |
    R^n 82 | nonterminal 83 | importance weight 84 (normalised by the batch max here) | p 85."""

    def __init__(self, capacity, stride=1, n_step=3, discount=0.99, priority_weight=0.4, priority_exponent=0.5,
                 deferred=False, device="cuda"):
        _abi.lib()
        self.device = torch.device(device)
        self.stride = int(stride)
        self.capacity = (int(capacity) // self.stride) * self.stride
        P = 1 << (self.capacity - 1).bit_length()
        if self.capacity < 2 or P > (1 << 22):
            raise ValueError(f"DevicePER capacity {capacity} (stride {stride}) outside [2, 2^22]")
        self.tree_leaves = P
        self.n_step, self.discount = int(n_step), float(discount)
        self.priority_weight, self.priority_exponent = float(priority_weight), float(priority_exponent)
        dev = self.device
        self.rows = torch.zeros((self.capacity, _abi.PER_DIM), dtype=torch.float32, device=dev)
        self.tree = torch.zeros(2 * P - 1, dtype=torch.float32, device=dev)
        self.state = torch.zeros(4, dtype=torch.int64, device=dev)
        self.t = torch.zeros(self.stride, dtype=torch.int32, device=dev)
        self.maxp = torch.ones(1, dtype=torch.float32, device=dev)
        self._weights = {}   # B -> the draws' contiguous weights (asvrl_per_sample_ex -> asvrl_per_normalise)
        self.dirty = torch.zeros(max(1, P // 2048), dtype=torch.uint8, device=dev)
        s = _abi.AsvPer()
        s.rows, s.tree, s.state, s.t = self.rows.data_ptr(), self.tree.data_ptr(), self.state.data_ptr(), \
            self.t.data_ptr()
        s.maxp, s.dirty = self.maxp.data_ptr(), self.dirty.data_ptr()
        s.capacity, s.tree_leaves, s.stride, s.n_step = self.capacity, P, self.stride, self.n_step
        s.discount, s.priority_weight, s.priority_exponent = self.discount, self.priority_weight, \
            self.priority_exponent
        s.deferred = 1 if deferred else 0
        self.deferred = bool(deferred)
        self._s = s
        self.pushed = 0   # host count of pushed slots (num_elements without a device sync)

    def push(self, obs, obj_cnt, actions, reward, done, stream=None, step_counter=None):
        """append() for n = m * stride rows (time-major); rows with obj_cnt < 0 become blank slots.
        step_counter: a device int64 [1] advanced by one in the push's last launch (asvrl_per_push_ex)."""
        n = obs.shape[0]
        adim = actions.shape[1] if actions.dim() == 2 else 1
        rc = _abi.lib().asvrl_per_push_ex(C.byref(self._s), _abi.ptr(obs), _abi.ptr(obj_cnt), _abi.ptr(actions),
                                          adim, _abi.ptr(reward), _abi.ptr(done), n, _abi.ptr(step_counter),
                                          _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_per_push")
        self.pushed += n

    def num_elements(self):
        """SegmentTree.num_elements (:62-66) from the host count (index + 1 until full)."""
        return self.capacity if self.pushed >= self.capacity else self.pushed + 1

    def sample(self, B, uniforms=None, seed=0, counter=0, counter_dev=None, out=None, out_idx=None, stream=None,
               normalise=True):
        out = out if out is not None else torch.empty((B, TR_DIM), dtype=torch.float32, device=self.device)
        assert out.shape[0] >= B and out.stride(0) == TR_DIM and out.stride(1) == 1, "rows [B][TR_DIM], contiguous"
        idx = out_idx if out_idx is not None else torch.empty(B, dtype=torch.int64, device=self.device)
        if uniforms is not None:
            uniforms = uniforms.to(device=self.device, dtype=torch.float64).contiguous()
        w = None
        if normalise:   # the draws' weights also contiguous, for the normalisation launch
            w = self._weights.get(B)
            if w is None:
                w = self._weights[B] = torch.empty(B, dtype=torch.float32, device=self.device)
        rc = _abi.lib().asvrl_per_sample_ex(C.byref(self._s), int(B), _abi.ptr(uniforms),
                                            int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF,
                                            _abi.ptr(counter_dev), _abi.ptr(out), _abi.ptr(idx), _abi.ptr(w),
                                            _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_per_sample")
        if normalise:   # weights / weights.max() (:191), one launch
            _abi.check(_abi.lib().asvrl_per_normalise(_abi.ptr(out), _abi.ptr(w), int(B), _abi.stream_ptr(stream)),
                       "asvrl_per_normalise")
        return out, idx

    def update_priorities(self, tree_idx, values, raw=False, stream=None, mean_out=None, learn_counter=None):
        """mean_out: f32 [1] receives values' mean, learn_counter: int64 [1] advanced by one, both in the update's
        last launch (asvrl_per_update_ex)."""
        v = values.detach().float().reshape(-1).contiguous()
        rc = _abi.lib().asvrl_per_update_ex(C.byref(self._s), _abi.ptr(tree_idx), _abi.ptr(v), v.shape[0],
                                            1 if raw else 0, _abi.ptr(mean_out), _abi.ptr(learn_counter),
                                            _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_per_update")

    def anomalies(self):
        return int(self.state[3].item())
