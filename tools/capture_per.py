#!/usr/bin/env python3
"""Capture golden vectors of Rainbow's prioritised replay from the reference (test infrastructure).

Runs ONLY in the build container, where the read-only reference is mounted at /root/reference:
it drives the reference's own ReplayMemory (rfarl/rfarl/policy/replay_memory_rainbow.py:98-196)
through a fixed append / sample / update_priorities sequence and writes tests/golden/per_memory.npz.
Nothing in the product, the GPU tests, smoke() or bench.py reads /root/reference.

    PYTHONDONTWRITEBYTECODE=1 python3 -W ignore tools/capture_per.py

Sequence: capacity 256, 640 appends of synthetic transitions (0..5 objects, 25 actions, terminal
with p = 0.08), a sample(32) + update_priorities after appends 300, 470 and 640 (the ring has
wrapped twice by the end). Recorded per event: the U(0,1) draws of the accepted stratified sample,
the sum tree before the sample, the sample's outputs, the priorities passed in, the resulting
np.power values, the tree and SegmentTree.max after the update.
"""
import os
import sys

import numpy as np

REF = "/root/reference/rfarl"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "per_memory.npz")
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

import torch  # noqa: E402
import rfarl.policy.replay_memory_rainbow as rm  # noqa: E402

CAP, B = 256, 32
EVENTS = (300, 470, 640)


class _Recorder:
    """np.random.uniform stand-in: low + (high - low) * random_sample(size), numpy's legacy uniform
    bit for bit, recording the U draws of the last call."""

    def __init__(self):
        self.last_u = None
        self.orig = np.random.uniform

    def __call__(self, low, high, size):
        u = np.random.random_sample(size)
        self.last_u = u
        return low + (float(high) - low) * u


def main():
    rng = np.random.RandomState(7)
    rec = _Recorder()
    np.random.uniform = rec
    mem = rm.ReplayMemory("cpu", CAP)
    n_total = EVENTS[-1]
    self_s = rng.uniform(-3, 3, size=(n_total, 7))
    n_obj = rng.randint(0, 6, size=n_total)
    objs = rng.uniform(-5, 5, size=(n_total, 5, 5))
    actions = rng.randint(0, 25, size=n_total)
    rewards = rng.uniform(-1.5, 1.5, size=n_total)
    terminal = rng.uniform(size=n_total) < 0.08
    out = dict(capacity=np.int64(CAP), batch=np.int64(B), events=np.array(EVENTS), self_s=self_s, n_obj=n_obj,
               objs=objs, actions=actions, rewards=rewards, terminal=terminal)
    np.random.seed(1234)
    k = 0
    for ev, upto in enumerate(EVENTS):
        while k < upto:
            st = (list(self_s[k]), [list(objs[k, j]) for j in range(n_obj[k])])
            mem.append(st, int(actions[k]), float(rewards[k]), bool(terminal[k]))
            k += 1
        out[f"e{ev}_tree_before"] = mem.transitions.sum_tree.copy()
        out[f"e{ev}_index"] = np.int64(mem.transitions.index)
        out[f"e{ev}_full"] = np.bool_(mem.transitions.full)
        out[f"e{ev}_t"] = np.int64(mem.t)
        idxs, s, a, R, ns, nt, w = mem.sample(B)
        out[f"e{ev}_u"] = rec.last_u.copy()
        out[f"e{ev}_tree_idx"] = np.asarray(idxs, np.int64)
        out[f"e{ev}_self"] = s[0].numpy()
        out[f"e{ev}_objs"] = s[1].numpy()
        out[f"e{ev}_mask"] = s[2].numpy()
        out[f"e{ev}_nself"] = ns[0].numpy()
        out[f"e{ev}_nobjs"] = ns[1].numpy()
        out[f"e{ev}_nmask"] = ns[2].numpy()
        out[f"e{ev}_action"] = a.numpy()
        out[f"e{ev}_R"] = R.numpy()
        out[f"e{ev}_nonterminal"] = nt.numpy()
        out[f"e{ev}_weights"] = w.numpy()
        loss = np.float32(rng.uniform(0.05, 4.0, size=B))
        out[f"e{ev}_loss"] = loss
        out[f"e{ev}_prio"] = np.power(loss, mem.priority_exponent)
        mem.update_priorities(idxs, loss)
        out[f"e{ev}_tree_after"] = mem.transitions.sum_tree.copy()
        out[f"e{ev}_max"] = np.float32(mem.transitions.max)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    torch.manual_seed(0)
    main()
