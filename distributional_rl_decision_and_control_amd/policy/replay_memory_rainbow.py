"""Prioritised n-step replay for Rainbow -- drop-in for rfarl.policy.replay_memory_rainbow
(replay_memory_rainbow.py:7-218).

Host-side sum tree over a structured transition array, with the reference's sampling rules:
one stratified draw per segment (np.random.uniform), rejection of indices too close to the
write head, n-step returns truncated at episode starts (timestep == 0), importance weights
(capacity * p)^-beta normalised by the batch max, priorities = loss^omega. Sampled batches
are moved to the device in one copy per field. (The device-resident PER is the next row of
SURVEY.md section 8f.)
"""
import numpy as np
import torch

TRANSITION = np.dtype([("timestep", np.int32), ("self_state", np.float32, (7,)),
                       ("object_states", np.float32, (5, 5)), ("object_state_masks", np.float32, (5,)),
                       ("action", np.int32), ("reward", np.float32), ("nonterminal", np.bool_)])
BLANK = (0, np.zeros((7,)), np.zeros((5, 5)), np.zeros((5,)), 0, 0.0, False)


class SumTree:
    """Complete binary sum tree with all leaves on the last level (replay_memory_rainbow.py:14-97)."""

    def __init__(self, size):
        self.index = 0
        self.size = size
        self.full = False
        self.tree_start = 2 ** (size - 1).bit_length() - 1
        self.sum_tree = np.zeros((self.tree_start + self.size,), dtype=np.float32)
        self.data = np.array([BLANK] * size, dtype=TRANSITION)
        self.max = 1

    def _refresh(self, nodes):
        kids = nodes * 2 + np.expand_dims([1, 2], axis=1)
        self.sum_tree[nodes] = np.sum(self.sum_tree[kids], axis=0)

    def _propagate(self, idx):
        parents = (idx - 1) // 2
        self._refresh(np.unique(parents))
        if parents[0] != 0:
            self._propagate(parents)

    def _propagate_one(self, i):
        parent = (i - 1) // 2
        self.sum_tree[parent] = self.sum_tree[2 * parent + 1] + self.sum_tree[2 * parent + 2]
        if parent != 0:
            self._propagate_one(parent)

    def update(self, indices, values):
        self.sum_tree[indices] = values
        self._propagate(indices)
        self.max = max(np.max(values), self.max)

    def append(self, data, value):
        self.data[self.index] = data
        self.sum_tree[self.index + self.tree_start] = value
        self._propagate_one(self.index + self.tree_start)
        self.max = max(value, self.max)
        self.index = (self.index + 1) % self.size
        self.full = self.full or self.index == 0
        self.max = max(value, self.max)

    def num_elements(self):
        return self.size if self.full else self.index + 1

    def _descend(self, idx, values):
        kids = idx * 2 + np.expand_dims([1, 2], axis=1)
        if kids[0, 0] >= self.sum_tree.shape[0]:
            return idx
        if kids[0, 0] >= self.tree_start:
            kids = np.minimum(kids, self.sum_tree.shape[0] - 1)
        left = self.sum_tree[kids[0]]
        go_right = np.greater(values, left).astype(np.int32)
        nxt = kids[go_right, np.arange(idx.size)]
        return self._descend(nxt, values - go_right * left)

    def find(self, values):
        idx = self._descend(np.zeros(values.shape, dtype=np.int32), values)
        return self.sum_tree[idx], idx - self.tree_start, idx

    def get(self, data_index):
        return self.data[data_index % self.size]

    def total(self):
        return self.sum_tree[0]


SegmentTree = SumTree  # reference name


class ReplayMemory:
    def __init__(self, device, capacity):
        self.device = device
        self.capacity = capacity
        self.history = 1
        self.discount = 0.99
        self.n = 3
        self.priority_weight = 0.4
        self.priority_exponent = 0.5
        self.t = 0
        self.n_step_scaling = torch.tensor([self.discount ** i for i in range(self.n)], dtype=torch.float32,
                                           device=self.device)
        self.transitions = SumTree(capacity)

    def state_batch(self, states):
        selfs = [s[0] for s in states]
        objs = [s[1] for s in states]
        if max(len(o) for o in objs) == 0:
            return selfs, [], []
        return (selfs, [o + [[0.] * 5] * (5 - len(o)) for o in objs],
                [[1.] * len(o) + [0.] * (5 - len(o)) for o in objs])

    def append(self, state, action, reward, terminal):
        """Stores (s_t, a_t) with r_{t+1}, terminal_{t+1} at max priority (replay_memory_rainbow.py:132-139)."""
        k = len(state[1])
        objects = np.array(state[1] + [[0., 0., 0., 0., 0.]] * (5 - k))
        masks = np.array([1.] * k + [0.] * (5 - k))
        self.transitions.append((self.t, np.array(state[0]), objects, masks, action, reward, not terminal),
                                self.transitions.max)
        self.t = 0 if terminal else self.t + 1

    def _window(self, idxs):
        """Transitions t-h+1 .. t+n with blanks across episode starts."""
        tr = self.transitions.get(np.arange(-self.history + 1, self.n + 1) + np.expand_dims(idxs, axis=1))
        firsts = tr["timestep"] == 0
        blank = np.zeros_like(firsts, dtype=np.bool_)
        for t in range(self.history - 2, -1, -1):
            blank[:, t] = np.logical_or(blank[:, t + 1], firsts[:, t + 1])
        for t in range(self.history, self.history + self.n):
            blank[:, t] = np.logical_or(blank[:, t - 1], firsts[:, t])
        tr[blank] = BLANK
        return tr

    def _draw(self, batch_size, p_total):
        seg = p_total / batch_size
        starts = np.arange(batch_size) * seg
        while True:
            samples = np.random.uniform(0.0, seg, [batch_size]) + starts
            probs, idxs, tree_idxs = self.transitions.find(samples)
            if (np.all((self.transitions.index - idxs) % self.capacity > self.n)
                    and np.all((idxs - self.transitions.index) % self.capacity >= self.history)
                    and np.all(probs != 0)):
                return probs, idxs, tree_idxs

    def sample(self, batch_size):
        p_total = self.transitions.total()
        probs, idxs, tree_idxs = self._draw(batch_size, p_total)
        tr = self._window(idxs)
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        h, n = self.history, self.n
        states = (torch.tensor(tr["self_state"][:, 0], **f32), torch.tensor(tr["object_states"][:, 0], **f32),
                  torch.tensor(tr["object_state_masks"][:, 0], **f32))
        next_states = (torch.tensor(tr["self_state"][:, n], **f32), torch.tensor(tr["object_states"][:, n], **f32),
                       torch.tensor(tr["object_state_masks"][:, n], **f32))
        actions = torch.tensor(np.copy(tr["action"][:, h - 1]), dtype=torch.int64, device=dev)
        rewards = torch.tensor(np.copy(tr["reward"][:, h - 1:-1]), **f32)
        R = torch.matmul(rewards, self.n_step_scaling)
        nonterminals = torch.tensor(np.expand_dims(tr["nonterminal"][:, h + n - 1], axis=1), **f32)
        probs = probs / p_total
        capacity = self.capacity if self.transitions.full else self.transitions.index
        weights = (capacity * probs) ** -self.priority_weight
        weights = torch.tensor(weights / weights.max(), **f32)
        return tree_idxs, states, actions, R, next_states, nonterminals, weights

    def update_priorities(self, idxs, priorities):
        self.transitions.update(idxs, np.power(priorities, self.priority_exponent))
