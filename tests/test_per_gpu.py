"""GPU: the HBM prioritised replay (asvrl_per_*, DevicePER) against the reference's captured
sequence (tests/golden/per_memory.npz) and the numpy oracle (oracle/per_oracle.py).

Bars: sum tree, sampled indices, observations, actions, nonterminal masks bit-exact; R^n within
1e-6 (CPU sgemv vs the kernel's ordered f32 sum); importance weights within 4e-6 rel. (device powf
vs numpy's SIMD powf); exponentiated priorities within 1 ulp (correctly rounded sqrt vs numpy's
powf(x, 0.5))."""
import numpy as np
import pytest
import torch

from oracle.per_oracle import PerOracle

pytestmark = pytest.mark.gpu


def _pack(g, lo, hi):
    from tests.test_per_golden import packed_obs
    return packed_obs(g, lo, hi)


def _push(per, obs, valid, actions, rewards, terminal):
    dev = per.device
    per.push(torch.from_numpy(obs).to(dev), torch.from_numpy(np.where(valid, 1, -1).astype(np.int8)).to(dev),
             torch.from_numpy(np.asarray(actions, np.float64).reshape(-1, 1)).to(dev),
             torch.from_numpy(np.asarray(rewards, np.float64)).to(dev),
             torch.from_numpy(np.asarray(terminal, np.uint8)).to(dev))


def full_tree(leaves, P):
    """Every level as pairwise f32 sums of the level below (the reference's node rule)."""
    lv = np.zeros(P, np.float32)
    lv[:leaves.size] = leaves
    levels = [lv]
    while lv.size > 1:
        lv = lv[0::2] + lv[1::2]
        levels.append(lv)
    return np.concatenate(levels[::-1])


def test_per_matches_reference_sequence():
    from distributional_rl_decision_and_control_amd.learn_ops import DevicePER
    from tests.test_per_golden import golden_sample
    g = dict(np.load("tests/golden/per_memory.npz"))
    cap, B = int(g["capacity"]), int(g["batch"])
    per = DevicePER(cap, stride=1, device="cuda")
    k = 0
    for ev, upto in enumerate(g["events"]):
        upto = int(upto)
        while k < upto:                     # pushes of <= capacity rows
            hi = min(upto, k + 200)
            _push(per, _pack(g, k, hi), np.ones(hi - k, bool), g["actions"][k:hi], g["rewards"][k:hi],
                  g["terminal"][k:hi])
            k = hi
        torch.cuda.synchronize()
        np.testing.assert_array_equal(per.tree.cpu().numpy(), g[f"e{ev}_tree_before"])
        st = per.state.cpu().numpy()
        assert st[0] == g[f"e{ev}_index"] and bool(st[1]) == bool(g[f"e{ev}_full"])
        assert per.t.cpu().numpy()[0] == g[f"e{ev}_t"]
        rows, idx = per.sample(B, uniforms=torch.from_numpy(g[f"e{ev}_u"]))
        rows, idx = rows.cpu().numpy(), idx.cpu().numpy()
        assert per.anomalies() == 0
        gs = golden_sample(g, ev)
        np.testing.assert_array_equal(idx, g[f"e{ev}_tree_idx"])
        np.testing.assert_array_equal(rows[:, 0:37], gs["obs"])
        np.testing.assert_array_equal(rows[:, 40:77], gs["next_obs"])
        np.testing.assert_array_equal(rows[:, 80], g[f"e{ev}_action"])
        np.testing.assert_allclose(rows[:, 82], g[f"e{ev}_R"], rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(rows[:, 83], g[f"e{ev}_nonterminal"].ravel())
        np.testing.assert_allclose(rows[:, 84], g[f"e{ev}_weights"], rtol=4e-6, atol=0)
        # exponentiation on the device: within 1 ulp of numpy's; then the exact update path
        snap = per.tree.clone(), per.maxp.clone(), per.dirty.clone()
        per.update_priorities(torch.from_numpy(idx).cuda(), torch.from_numpy(g[f"e{ev}_loss"]).cuda())
        ti = g[f"e{ev}_tree_idx"]
        want = g[f"e{ev}_tree_before"].copy()
        want[ti] = g[f"e{ev}_prio"]          # duplicates: the last occurrence wins
        ulp = np.abs(per.tree.cpu().numpy()[ti].view(np.int32) - want[ti].view(np.int32))
        assert ulp.max() <= 1
        per.tree.copy_(snap[0]), per.maxp.copy_(snap[1]), per.dirty.copy_(snap[2])
        per.update_priorities(torch.from_numpy(idx).cuda(), torch.from_numpy(g[f"e{ev}_prio"]).cuda(), raw=True)
        np.testing.assert_array_equal(per.tree.cpu().numpy(), g[f"e{ev}_tree_after"])
        assert per.maxp.item() == g[f"e{ev}_max"]


@pytest.mark.parametrize("stride,cap,B,deferred", [(40, 40 * 96, 16, False), (1000, 1000 * 40, 8, False),
                                                   (40, 40 * 96, 256, True), (1000, 1000 * 40, 4096, True)])
def test_per_strided_matches_oracle(stride, cap, B, deferred):
    """One stream per robot (stride = envs x robots): pushes with blank slots, wrap-around, samples
    and priority updates agree with the numpy restatement."""
    from distributional_rl_decision_and_control_amd.learn_ops import DevicePER
    rng = np.random.RandomState(stride)
    per = DevicePER(cap, stride=stride, deferred=deferred, device="cuda")
    o = PerOracle(cap, stride=stride, deferred=deferred)
    steps = cap // stride + cap // stride // 2
    checked = 0
    for step in range(steps):
        obs = rng.uniform(-2, 2, size=(stride, 40)).astype(np.float32)
        valid = rng.uniform(size=stride) > 0.1
        act = rng.randint(0, 25, size=stride)
        rew = rng.uniform(-1, 1, size=stride)
        term = rng.uniform(size=stride) < 0.05
        _push(per, obs, valid, act, rew, term)
        o.push(obs, valid, act, rew, term)
        if step % 7 == 6:
            torch.cuda.synchronize()
            np.testing.assert_array_equal(per.tree.cpu().numpy(), o.tree)
            for attempt in range(200):  # the reference redraws the whole batch until it is valid
                u = rng.uniform(size=B)
                ref = o.sample(B, u)
                if ref is not None:
                    break
                assert not deferred     # deferred trees hold only complete windows: never rejects
            if ref is None:
                continue
            rows, idx = per.sample(B, uniforms=torch.from_numpy(u))
            rows, idx = rows.cpu().numpy(), idx.cpu().numpy()
            np.testing.assert_array_equal(idx, ref["tree_idx"])
            np.testing.assert_array_equal(rows[:, 0:40], ref["obs"])
            np.testing.assert_array_equal(rows[:, 40:80], ref["next_obs"])
            np.testing.assert_array_equal(rows[:, 80], ref["action"])
            np.testing.assert_allclose(rows[:, 82], ref["R"], rtol=1e-6, atol=1e-6)
            np.testing.assert_array_equal(rows[:, 83], ref["nonterminal"])
            np.testing.assert_allclose(rows[:, 84], ref["weights"], rtol=4e-6)
            prio = np.float32(rng.uniform(0.01, 3.0, size=B))
            per.update_priorities(torch.from_numpy(idx).cuda(), torch.from_numpy(prio).cuda(), raw=True)
            o.update(ref["tree_idx"], prio)
            checked += 1
    torch.cuda.synchronize()
    np.testing.assert_array_equal(per.tree.cpu().numpy(), o.tree)
    assert per.maxp.item() == np.float32(o.max)
    assert per.anomalies() == 0 and checked >= 2


def test_per_full_size_tree_and_sampling():
    """Bench shape: 8192 envs x 5 robots per push, 4,096,000 slots (2^22 leaves, 2048 subtree
    blocks + the top kernel). The tree equals the level-by-level f32 rebuild from its leaves; Philox
    samples are valid (p > 0, behind the head, sorted), and a large leaf is drawn in proportion."""
    from distributional_rl_decision_and_control_amd.learn_ops import DevicePER
    S = 8192 * 5
    per = DevicePER(S * 100, stride=S, deferred=True, device="cuda")
    assert per.tree_leaves == 1 << 22
    g = torch.Generator(device="cuda").manual_seed(0)
    for step in range(6):
        obs = torch.rand((S, 40), device="cuda", generator=g)
        cnt = torch.where(torch.rand(S, device="cuda", generator=g) > 0.2, 1, -1).to(torch.int8)
        act = torch.randint(0, 25, (S, 1), device="cuda", generator=g).double()
        rew = torch.rand(S, device="cuda", generator=g).double()
        done = (torch.rand(S, device="cuda", generator=g) < 0.05).to(torch.uint8)
        per.push(obs, cnt, act, rew, done)
    B = 8192
    rows, idx = per.sample(B, seed=5, counter=1)
    # priorities: spread over [0.1, 10]
    per.update_priorities(idx, torch.rand(B, device="cuda", generator=g) * 100 + 0.01)
    torch.cuda.synchronize()
    P = per.tree_leaves
    t = per.tree.cpu().numpy()
    np.testing.assert_array_equal(t, full_tree(t[P - 1:P - 1 + per.capacity], P))
    rows, idx = per.sample(B, seed=5, counter=2)
    torch.cuda.synchronize()
    idx = idx.cpu().numpy()
    assert per.anomalies() == 0
    assert np.all(np.diff(idx) >= 0)
    leaves = t[idx]
    assert np.all(leaves > 0)
    di = idx - (P - 1)
    assert np.all(di < 6 * S - 3 * S)          # only complete windows are in the tree
    r = rows.cpu().numpy()
    assert np.all(r[:, 84] <= 1.0) and r[:, 84].max() == 1.0
    # proportional: the share of draws landing on the top-1% priority leaves tracks their mass
    live = t[P - 1:P - 1 + 3 * S]
    thr = np.quantile(live[live > 0], 0.99)
    mass = live[live >= thr].sum() / live.sum()
    share = np.mean(leaves >= thr)
    assert abs(share - mass) < 0.1 * mass + 0.01


def test_vec_trainer_rainbow_graph():
    """The batched Rainbow loop (act_rainbow on every robot, env step, PER push, sample, train_Rainbow
    on the C51 kernel, update_priorities) under HIP-graph replay: finite losses, the sampled
    leaves' priorities become loss**0.5, no PER anomalies, the online weights move."""
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    tr = VecTrainer(n_envs=128, agent_type="Rainbow", batch_size=256, buffer_size=128 * 5 * 40, graphs=True,
                    seed=3)
    w0 = tr.local.hidden_layer_a.weight_mu.detach().clone()
    n = 0
    while tr.replay_size_host() < tr.learning_starts:
        tr.iteration()
        n += 1
    assert n >= tr.n_step + 1
    losses = []
    for _ in range(8):
        out = tr.iteration()
        losses.append(out[0].item())
    torch.cuda.synchronize()
    assert all(np.isfinite(losses)) and tr.per.anomalies() == 0
    idx = tr.per_idx.cpu().numpy()
    assert np.all(np.diff(idx) >= 0)
    assert not torch.equal(w0, tr.local.hidden_layer_a.weight_mu.detach())
    assert tr.per.tree[0].item() > 0


def test_per_unvalidated_draw_gets_zero_weight():
    """A draw that never validates (here: the injected uniform of the last segment lands on a
    transition whose n-step window reaches the write head, replay_memory_rainbow.py:163) is counted
    as an anomaly and gets importance weight 0, so it cannot turn w / w.max() into NaN."""
    from distributional_rl_decision_and_control_amd.learn_ops import DevicePER
    rng = np.random.RandomState(5)
    per = DevicePER(256, stride=1, device="cuda")
    n = 100
    obs = rng.randn(n, 40).astype(np.float32)
    _push(per, obs, np.ones(n, bool), rng.randint(0, 25, n), rng.randn(n), np.zeros(n, np.uint8))
    B = 32
    u = np.full(B, 0.5)
    u[B - 1] = 0.999
    rows, idx = per.sample(B, uniforms=torch.from_numpy(u))
    rows = rows.cpu().numpy()
    torch.cuda.synchronize()
    assert per.anomalies() == 1
    w = rows[:, 84]
    assert np.all(np.isfinite(w)) and w[B - 1] == 0.0 and np.all(w[:B - 1] > 0) and np.isclose(w.max(), 1.0)
    # the unvalidated draw is marked -1 and update_priorities leaves its leaf as it was
    ix = idx.cpu().numpy()
    assert ix[B - 1] == -1 and np.all(ix[:B - 1] >= 0)
    leaf = per.tree_leaves - 1 + int(rows[B - 1, 86])
    before = per.tree.clone()
    per.update_priorities(idx, torch.full((B,), 4.0, device="cuda"))
    torch.cuda.synchronize()
    assert per.tree[leaf].item() == before[leaf].item()
    assert per.anomalies() == 1   # the -1 entry is not an ordering anomaly
    assert np.all(per.tree[torch.from_numpy(ix[:B - 1]).cuda()].cpu().numpy() == 2.0)


def test_per_fused_tail_work():
    """ABI 25: asvrl_per_sample_ex + asvrl_per_normalise (weights / weights.max() in one launch) equal torch's
    w.div_(w.max()) bit for bit; asvrl_per_update_ex's values mean (fixed order) equals the mean within f32 rounding and it advances the
    learn counter by one; asvrl_per_push_ex advances the step counter by one. The batched Rainbow loop then counts
    exactly one env step per iteration and one learn step per learning iteration (eager)."""
    from distributional_rl_decision_and_control_amd.learn_ops import DevicePER
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    S = 640
    per = DevicePER(S * 20, stride=S, deferred=True, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    for step in range(6):
        obs = torch.rand((S, 40), device="cuda", generator=g)
        cnt = torch.ones(S, dtype=torch.int8, device="cuda")
        act = torch.randint(0, 25, (S, 1), device="cuda", generator=g).double()
        rew = torch.rand(S, device="cuda", generator=g).double()
        done = (torch.rand(S, device="cuda", generator=g) < 0.05).to(torch.uint8)
        per.push(obs, cnt, act, rew, done, step_counter=ctr)
    assert int(ctr.item()) == 6
    B = 1000
    rows, idx = per.sample(B, seed=3, counter=1, normalise=False)
    w = rows[:, 84].clone()
    w.div_(w.max())
    rows2, idx2 = per.sample(B, seed=3, counter=1)   # the same draws, normalised by asvrl_per_normalise
    torch.cuda.synchronize()
    assert torch.equal(idx2, idx) and torch.equal(rows2[:, 84], w) and torch.equal(rows2[:, :84], rows[:, :84])
    vals = torch.rand(B, device="cuda", generator=g) * 3
    mean = torch.zeros(1, device="cuda")
    lc = torch.full((1,), 41, dtype=torch.int64, device="cuda")
    per.update_priorities(idx, vals, mean_out=mean, learn_counter=lc)
    torch.cuda.synchronize()
    assert int(lc.item()) == 42
    assert abs(float(mean.item()) - float(vals.double().mean().item())) <= 1e-6 * float(vals.double().mean().item())
    tr = VecTrainer(n_envs=64, agent_type="Rainbow", batch_size=128, buffer_size=64 * 5 * 40, graphs=False, seed=4)
    c0, l0, k, learned = int(tr.env.counter.item()), int(tr.learn_counter.item()), 0, 0
    while learned < 3:
        out = tr.iteration()
        k += 1
        learned += out is not None
    torch.cuda.synchronize()
    assert int(tr.env.counter.item()) == c0 + k
    assert int(tr.learn_counter.item()) == l0 + learned
    assert np.isfinite(float(out[0].item()))
