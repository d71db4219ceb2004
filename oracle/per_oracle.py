"""CPU restatement of Rainbow's prioritised n-step replay -- TEST INFRASTRUCTURE ONLY.

Imported by tests/ (and nothing in the product path). It restates the reference's ReplayMemory +
SegmentTree (rfarl/rfarl/policy/replay_memory_rainbow.py:14-196) in numpy, generalised to
`stride` slots per time step exactly as the device ring (asvrl_per.hip) is: the n-step window of
slot i is i, i + stride, ..., i + n*stride; stride = 1 is the reference itself. `deferred`
restates the device's batched mode: an append's priority enters the tree when the append n steps
later completes its window (asvrl_per.hip header), and the head-slot rule is dropped. Pinned at
stride 1 against tests/golden/per_memory.npz (captured from the reference by
tools/capture_per.py) in tests/test_oracle_golden.py.
"""
import numpy as np

PER_ROW = np.dtype([("timestep", np.int32), ("obs", np.float32, (40,)), ("action", np.int32),
                    ("reward", np.float32), ("nonterminal", np.bool_)])


class PerOracle:
    def __init__(self, capacity, stride=1, n=3, discount=0.99, priority_weight=0.4, priority_exponent=0.5,
                 deferred=False):
        self.deferred = bool(deferred)
        self.capacity, self.stride, self.n = int(capacity), int(stride), int(n)
        self.discount, self.beta, self.omega = discount, priority_weight, priority_exponent
        self.P = 1 << (self.capacity - 1).bit_length()          # tree_start + 1 (:17)
        self.tree = np.zeros(2 * self.P - 1, np.float32)
        self.data = np.zeros(self.capacity, PER_ROW)
        self.index, self.full, self.max = 0, False, 1
        self.t = np.zeros(self.stride, np.int64)                 # ReplayMemory.t per stream (:107)
        self.prio = np.zeros(self.capacity, np.float32)          # append priority kept per slot
        self.scaling = np.array([discount ** i for i in range(n)], np.float32)  # n_step_scaling (:108)

    # ---------------------------------------------------------------- SegmentTree (:14-97)
    def _propagate_index(self, i):                               # :36-41
        while i != 0:
            p = (i - 1) // 2
            self.tree[p] = self.tree[2 * p + 1] + self.tree[2 * p + 2]
            i = p

    def _find(self, values):                                     # :72-91
        idx = np.zeros(values.shape, np.int64)
        last = self.P - 1 + self.capacity - 1
        while True:
            kids = idx * 2 + np.expand_dims([1, 2], axis=1)
            if kids[0, 0] >= self.tree.shape[0]:
                break
            if kids[0, 0] >= self.P - 1:
                kids = np.minimum(kids, last)
            left = self.tree[kids[0]]
            go = np.greater(values, left).astype(np.int32)
            idx = kids[go, np.arange(idx.size)]
            values = values - go * left
        return self.tree[idx], idx - (self.P - 1), idx

    # ---------------------------------------------------------------- ReplayMemory (:98-196)
    def push(self, obs, valid, actions, rewards, terminal):
        """m * stride rows, time-major: stream k % stride appends row k (append, :132-139) or a
        blank slot of priority 0 when not valid."""
        n = obs.shape[0]
        assert n % self.stride == 0
        for k in range(n):
            r = k % self.stride
            slot = (self.index + k) % self.capacity
            if valid[k]:
                self.data[slot] = (self.t[r], obs[k], int(actions[k]), np.float32(rewards[k]), not terminal[k])
                self.prio[slot] = self.max
                self.t[r] = 0 if terminal[k] else self.t[r] + 1
            else:
                self.data[slot] = (0, np.zeros(40), 0, 0.0, False)
                self.prio[slot] = 0.0
                self.t[r] = 0
            self.tree[self.P - 1 + slot] = 0.0 if self.deferred else self.prio[slot]
            self._propagate_index(self.P - 1 + slot)
            if self.deferred:
                act = (self.index + k - self.n * self.stride) % self.capacity
                self.tree[self.P - 1 + act] = self.prio[act]
                self._propagate_index(self.P - 1 + act)
        nx = self.index + n
        self.full = self.full or nx >= self.capacity
        self.index = nx % self.capacity

    def sample(self, B, u):
        """u: the U(0, 1) draws of one stratified attempt; returns None if the reference would redraw."""
        total = self.tree[0]
        seg = total / B
        samples = (0.0 + (float(seg) - 0.0) * u) + np.arange(B) * seg
        probs, idxs, tree_idxs = self._find(samples)
        S, C = self.stride, self.capacity
        if self.deferred:   # distance behind the head in [1, C]: the head slot holds the oldest data
            ok = np.all((self.index - idxs - 1) % C + 1 > self.n * S) and np.all(probs != 0)
        else:               # :163
            ok = (np.all((self.index - idxs) % C > self.n * S) and np.all((idxs - self.index) % C >= S)
                  and np.all(probs != 0))
        if not ok:
            return None
        win = self.data[(idxs[:, None] + S * np.arange(self.n + 1)[None, :]) % C]
        firsts = win["timestep"] == 0
        blank = np.zeros_like(firsts)
        for t in range(1, self.n + 1):
            blank[:, t] = np.logical_or(blank[:, t - 1], firsts[:, t])
        win[blank] = (0, np.zeros(40), 0, 0.0, False)
        R = win["reward"][:, :self.n].astype(np.float32) @ self.scaling
        p = probs / total
        cap = C if self.full else self.index
        w = (cap * p) ** -self.beta
        return dict(tree_idx=tree_idxs, data_idx=idxs, obs=win["obs"][:, 0], next_obs=win["obs"][:, self.n],
                    action=win["action"][:, 0], R=R, nonterminal=win["nonterminal"][:, self.n].astype(np.float32),
                    weights=w / w.max(), p=p)

    def update(self, tree_idxs, values):
        """update_priorities with values already exponentiated (:194-196, SegmentTree.update :44-53)."""
        self.tree[tree_idxs] = values
        for i in np.unique(tree_idxs):
            self._propagate_index(int(i))
        self.max = max(np.max(values), self.max)
