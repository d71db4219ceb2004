"""ReplayBuffer -- drop-in for rfarl.utils.replay_buffer.ReplayBuffer (replay_buffer.py:6-69).

Transitions live in an HBM ring (learn_ops.DeviceReplay) instead of a deque of Python
tuples. add() packs one (s, a, r, s', done) into the 88-float row on the host and stages
it; sample() flushes the staged rows with one copy + asvrl_replay_write_rows, draws the
batch indices with Python's `random.sample` exactly like the reference (so a seeded run
picks the same transitions), and gathers them on the device with asvrl_replay_sample.
"""
import random

import numpy as np
import torch

from .._abi import OBS_DIM, TR_DIM
from ..learn_ops import DeviceReplay, split_rows


def pack_state(state, obj_len=5, max_obj_num=5, out=None):
    """(self[7], objects[<=5][5]) -> packed f32 row: self | objects padded | mask (state_batch)."""
    row = out if out is not None else np.zeros(OBS_DIM, np.float32)
    self_state, objects = state
    row[:7] = np.asarray(self_state, dtype=np.float64)
    k = len(objects)
    if k:
        row[7:7 + obj_len * k] = np.asarray(objects, dtype=np.float64).reshape(-1)
    row[7 + obj_len * k:7 + obj_len * max_obj_num] = 0.0
    row[32:32 + k] = 1.0
    row[32 + k:37] = 0.0
    return row


class ReplayBuffer:
    def __init__(self, buffer_size, batch_size, obj_len, max_object_num, seed=249, device="cuda"):
        self.capacity = int(buffer_size)
        self.batch_size = batch_size
        self.obj_len = obj_len
        self.max_obj_num = max_object_num
        self.seed = random.seed(seed)  # replay_buffer.py:20 (seeds Python's global RNG)
        self.device = torch.device(device)
        self.ring = DeviceReplay(self.capacity, device=self.device)
        self._count = 0          # transitions ever added
        self._staged = []        # host rows not yet on the device
        self._staged_slots = []

    def add(self, item):
        """replay_buffer.py:22-24."""
        s, a, r, ns, d = item
        row = np.zeros(TR_DIM, np.float32)
        pack_state(s, self.obj_len, self.max_obj_num, row[:OBS_DIM])
        pack_state(ns, self.obj_len, self.max_obj_num, row[OBS_DIM:2 * OBS_DIM])
        if isinstance(a, (list, tuple, np.ndarray)):
            av = np.asarray(a, dtype=np.float64).reshape(-1)
            row[80:80 + av.size] = av
        else:
            row[80] = float(a)
        row[82] = float(r)
        row[83] = float(bool(d))
        self._staged.append(row)
        self._staged_slots.append(self._count % self.capacity)
        self._count += 1

    def size(self):
        return min(self._count, self.capacity)

    def __len__(self):
        return self.size()

    def flush(self):
        if not self._staged:
            return
        rows = torch.from_numpy(np.stack(self._staged)).to(self.device)
        slots = torch.tensor(self._staged_slots, dtype=torch.int64, device=self.device)
        self.ring.write_rows(rows, slots)
        n = self.size()
        self.ring.state.copy_(torch.tensor([self._count % self.capacity, n], dtype=torch.int64))
        self._staged.clear()
        self._staged_slots.clear()

    def sample_rows(self):
        self.flush()
        idx = random.sample(range(self.size()), k=self.batch_size)  # replay_buffer.py:28
        return self.ring.gather(torch.tensor(idx, dtype=torch.int64, device=self.device))

    def sample(self):
        """replay_buffer.py:26-45 -> (states, actions, rewards, next_states, dones) as device
        tensors: states = (self (B,7), objects (B,5,5), mask (B,5)); rewards/dones (B,1)."""
        return split_rows(self.sample_rows())

    def state_batch(self, states):
        """replay_buffer.py:51-69 (host lists; used by Agent.act_* for batch-1 acting)."""
        self_state_batch = []
        object_states_batch = []
        for state in states:
            self_state_batch.append(state[0])
            object_states_batch.append(state[1])
        max_curr_obj_num = max(len(sublist) for sublist in object_states_batch)
        if max_curr_obj_num == 0:
            return self_state_batch, [], []
        padded = [sublist + [[0.] * self.obj_len] * (self.max_obj_num - len(sublist)) for sublist in object_states_batch]
        mask = [[1.] * len(sublist) + [0.] * (self.max_obj_num - len(sublist)) for sublist in object_states_batch]
        return self_state_batch, padded, mask
