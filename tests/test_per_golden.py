"""CPU: Rainbow's prioritised n-step replay (replay_memory_rainbow.py:14-196) pinned against the
reference's own outputs (tests/golden/per_memory.npz, tools/capture_per.py): the numpy oracle
(oracle/per_oracle.py, stride 1) and the drop-in host ReplayMemory reproduce every sample, weight
and sum-tree state of the captured sequence."""
import os

import numpy as np
import pytest

from oracle.per_oracle import PerOracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "per_memory.npz")


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLD))


def packed_obs(g, lo, hi):
    """The ASVRL_OBS_DIM rows (self 7 | objects 25 | mask 5 | pad 3) of appends lo..hi-1."""
    n = hi - lo
    o = np.zeros((n, 40), np.float32)
    o[:, :7] = g["self_s"][lo:hi]
    for k in range(n):
        c = int(g["n_obj"][lo + k])
        o[k, 7:7 + 5 * c] = g["objs"][lo + k, :c].reshape(-1)
        o[k, 32:32 + c] = 1.0
    return o


def golden_sample(g, ev):
    B = int(g["batch"])
    return dict(obs=np.concatenate([g[f"e{ev}_self"], g[f"e{ev}_objs"].reshape(B, 25), g[f"e{ev}_mask"]], 1),
                next_obs=np.concatenate([g[f"e{ev}_nself"], g[f"e{ev}_nobjs"].reshape(B, 25), g[f"e{ev}_nmask"]], 1))


def test_per_oracle_matches_reference(g):
    cap, B = int(g["capacity"]), int(g["batch"])
    o = PerOracle(cap, stride=1)
    k = 0
    for ev, upto in enumerate(g["events"]):
        obs = packed_obs(g, k, upto)
        o.push(obs, np.ones(upto - k, bool), g["actions"][k:upto], g["rewards"][k:upto], g["terminal"][k:upto])
        k = int(upto)
        np.testing.assert_array_equal(o.tree, g[f"e{ev}_tree_before"])
        assert o.index == g[f"e{ev}_index"] and o.full == g[f"e{ev}_full"] and o.t[0] == g[f"e{ev}_t"]
        s = o.sample(B, g[f"e{ev}_u"])
        assert s is not None
        gs = golden_sample(g, ev)
        np.testing.assert_array_equal(s["tree_idx"], g[f"e{ev}_tree_idx"])
        np.testing.assert_array_equal(s["obs"][:, :37], gs["obs"])
        np.testing.assert_array_equal(s["next_obs"][:, :37], gs["next_obs"])
        np.testing.assert_array_equal(s["action"], g[f"e{ev}_action"])
        np.testing.assert_allclose(s["R"], g[f"e{ev}_R"], rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(s["nonterminal"], g[f"e{ev}_nonterminal"].ravel())
        np.testing.assert_array_equal(s["weights"], g[f"e{ev}_weights"])
        o.update(s["tree_idx"], g[f"e{ev}_prio"])
        np.testing.assert_array_equal(o.tree, g[f"e{ev}_tree_after"])
        assert np.float32(o.max) == g[f"e{ev}_max"]


def test_host_replay_memory_matches_reference(g):
    """The drop-in ReplayMemory (Agent's Rainbow path) replays the captured sequence exactly."""
    from distributional_rl_decision_and_control_amd.policy.replay_memory_rainbow import ReplayMemory
    cap, B = int(g["capacity"]), int(g["batch"])
    mem = ReplayMemory("cpu", cap)
    state = np.random.get_state()
    np.random.seed(1234)
    try:
        k = 0
        for ev, upto in enumerate(g["events"]):
            while k < upto:
                c = int(g["n_obj"][k])
                st = (list(g["self_s"][k]), [list(g["objs"][k, j]) for j in range(c)])
                mem.append(st, int(g["actions"][k]), float(g["rewards"][k]), bool(g["terminal"][k]))
                k += 1
            np.testing.assert_array_equal(mem.transitions.sum_tree[:2 * cap - 1], g[f"e{ev}_tree_before"])
            idxs, s, a, R, ns, nt, w = mem.sample(B)
            np.testing.assert_array_equal(idxs, g[f"e{ev}_tree_idx"])
            np.testing.assert_array_equal(s[0].numpy(), g[f"e{ev}_self"])
            np.testing.assert_array_equal(ns[1].numpy(), g[f"e{ev}_nobjs"])
            np.testing.assert_array_equal(a.numpy(), g[f"e{ev}_action"])
            np.testing.assert_allclose(R.numpy(), g[f"e{ev}_R"], rtol=1e-6, atol=1e-6)
            np.testing.assert_array_equal(nt.numpy(), g[f"e{ev}_nonterminal"])
            np.testing.assert_array_equal(w.numpy(), g[f"e{ev}_weights"])
            mem.update_priorities(idxs, g[f"e{ev}_loss"])
            np.testing.assert_array_equal(mem.transitions.sum_tree[:2 * cap - 1], g[f"e{ev}_tree_after"])
    finally:
        np.random.set_state(state)


def test_per_oracle_stride_windows_stay_in_stream():
    """stride > 1: every window is one stream's own consecutive transitions, blanked at its episode
    starts, and blank (non-acting) slots are never sampled."""
    S, cap = 4, 64
    o = PerOracle(cap, stride=S)
    rng = np.random.RandomState(3)
    for step in range(30):
        obs = np.zeros((S, 40), np.float32)
        obs[:, 0] = np.arange(S)          # stream id
        obs[:, 1] = step                  # time
        valid = rng.uniform(size=S) > 0.1
        term = rng.uniform(size=S) < 0.15
        o.push(obs, valid, np.arange(S), np.full(S, 1.0), term)
    for trial in range(20):
        s = o.sample(8, rng.uniform(size=8))
        if s is None:
            continue
        np.testing.assert_array_equal(s["data_idx"] % S, s["obs"][:, 0])
        live = s["nonterminal"] > 0
        np.testing.assert_array_equal(s["next_obs"][live, 0], s["obs"][live, 0])
        np.testing.assert_array_equal(s["next_obs"][live, 1], s["obs"][live, 1] + 3)
        assert np.all(s["p"] > 0)
