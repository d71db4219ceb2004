"""GPU parity of the HAND-WRITTEN learner -- the kernels bench.py times -- against the reference's
own train_AC_IQN / train_IQN numbers (tests/golden/learn_ac_iqn.npz, learn_iqn.npz; captured by
tools/capture_oracle.py from rfarl/rfarl/agent.py:386-432,434-476).

fused_update.ac_iqn_update_fused2 and fused_iqn.iqn_update_fused run on the captured B = 64
batches with the captured tau draws injected, from the seeded initial weights:

  * operands "f32"  -- libasvrl_f32.so, the same kernel sources built with f32 operands
    (v_mfma_f32_32x32x2_f32): the reference's fp32 bar, losses within 1e-5 rel., pre-clip gradient
    norms within 1e-4 rel., weights after Adam steps 1 and 3 within 1e-4 rel. / 2e-6 abs. (the bar
    test_agent_gpu holds the torch learner to);
  * operands "bf16" -- libasvrl.so, the training build (bf16 MFMA operands, f32 accumulation):
    losses within 2e-2 rel., gradient norms within 5e-2 rel., and the Adam update (after - initial)
    with cosine > 0.97 to the reference's over the whole network, > 0.75 for every tensor (Adam's
    first steps are about +-lr per element, so bf16 noise on near-zero gradient elements flips
    single elements; the 56-element encoder bias sees it most, observed 0.84).

Plus one tracking test at the bench shape (B = 4096, N = 32): bf16 vs f32 builds of the same update
on the same random batch (losses 2e-2, update cosine > 0.95).
"""
import numpy as np
import pytest
import torch

from oracle import env_oracle as eo
from oracle import learn_ref as lr

pytestmark = pytest.mark.gpu

BARS = {"f32": dict(loss=1e-5, norm=1e-4), "bf16": dict(loss=2e-2, norm=5e-2)}


def _rows(z, p, discrete=False):
    """Replay rows [B][88] (obs | next obs | action | reward | done) of a captured batch."""
    B = z[p + "s_self"].shape[0]
    rows = np.zeros((B, 88), np.float32)
    for c, pre in ((0, "s_"), (40, "ns_")):
        rows[:, c:c + 7] = z[p + pre + "self"]
        rows[:, c + 7:c + 32] = z[p + pre + "obj"].reshape(B, 25)
        rows[:, c + 32:c + 37] = z[p + pre + "mask"]
    a = z[p + "a"].reshape(B, -1)
    rows[:, 80:80 + a.shape[1]] = a
    rows[:, 82] = z[p + "r"]
    rows[:, 83] = z[p + "d"]
    return torch.from_numpy(rows).cuda()


def _cos(x, y):
    x, y = x.reshape(-1).astype(np.float64), y.reshape(-1).astype(np.float64)
    return float(x @ y / (np.linalg.norm(x) * np.linalg.norm(y) + 1e-300))


def _check_params(module, z, prefix, before, ops):
    """f32: every parameter within 1e-4 rel. / 2e-6 abs. of the reference; bf16: the whole network's
    Adam update (after - initial) with cosine > 0.97 to the reference's, every tensor's > 0.75.
    Returns the worst per-tensor cosine."""
    worst, gd, rd = 1.0, [], []
    for k, v in module.state_dict().items():
        got, ref = v.detach().cpu().numpy(), z[prefix + k]
        if ops == "f32":
            np.testing.assert_allclose(got, ref, rtol=1e-4, atol=2e-6, err_msg=prefix + k)
        else:
            c = _cos(got - before[k], ref - before[k])
            worst = min(worst, c)
            assert c > 0.75, (prefix + k, c)
            gd.append((got - before[k]).reshape(-1))
            rd.append((ref - before[k]).reshape(-1))
    if gd:
        c = _cos(np.concatenate(gd), np.concatenate(rd))
        assert c > 0.97, (prefix, c)
    return worst


def _snapshot(module):
    return {k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def _ac_iqn(ops, B, N):
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    ag = Agent(seed=100, agent_type="AC-IQN")
    loc, tgt = ag.policy_local, ag.policy_target
    ao = FusedAdam(loc.actor.parameters(), lr=1e-4, operands=ops)
    co = FusedAdam(loc.critic.parameters(), lr=1e-4, operands=ops)
    st = FusedACIQNState(loc, tgt, B, N, operands=ops)
    return loc, tgt, ao, co, st


@pytest.mark.parametrize("ops", ["f32", "bf16"])
def test_fused_ac_iqn_matches_reference(ops):
    """Three train_AC_IQN steps (N = N' = 8), the fused kernels of the benched path."""
    from distributional_rl_decision_and_control_amd.fused_update import ac_iqn_update_fused2
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    loc, tgt, ao, co, st = _ac_iqn(ops, 64, 8)
    for k, v in loc.actor.state_dict().items():
        np.testing.assert_array_equal(v.cpu().numpy(), z["init/actor/" + k])
    bar = BARS[ops]
    before = {"actor": _snapshot(loc.actor), "critic": _snapshot(loc.critic)}
    for step in range(3):
        rows = _rows(z, f"step{step}/")
        taus = torch.from_numpy(z[f"step{step}/taus"][..., 0]).cuda().contiguous()
        cl, al, cgn, agn = ac_iqn_update_fused2(st, loc, ao, co, co.grads, ao.grads, rows, taus=taus)
        torch.cuda.synchronize()
        np.testing.assert_allclose(cl.item(), z[f"step{step}/critic_loss"], rtol=bar["loss"])
        np.testing.assert_allclose(al.item(), z[f"step{step}/actor_loss"], rtol=bar["loss"])
        np.testing.assert_allclose([cgn.item(), agn.item()], z[f"step{step}/grad_norms"], rtol=bar["norm"])
        if step in (0, 2):
            wa = _check_params(loc.actor, z, f"after{step}/actor/", before["actor"], ops)
            wc = _check_params(loc.critic, z, f"after{step}/critic/", before["critic"], ops)
            print(f"{ops} step {step}: losses {cl.item():.7g} {al.item():.7g}, worst update cosine {min(wa, wc):.4f}")


@pytest.mark.parametrize("ops", ["f32", "bf16"])
def test_fused_ac_iqn_32_quantiles_matches_reference(ops):
    """BASELINE config 2's N = N' = 32: one step on the captured batch."""
    from distributional_rl_decision_and_control_amd.fused_update import ac_iqn_update_fused2
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    loc, tgt, ao, co, st = _ac_iqn(ops, 64, 32)
    bar = BARS[ops]
    before = {"actor": _snapshot(loc.actor), "critic": _snapshot(loc.critic)}
    rows = _rows(z, "n32/")
    taus = torch.from_numpy(z["n32/taus"][..., 0]).cuda().contiguous()
    cl, al, cgn, agn = ac_iqn_update_fused2(st, loc, ao, co, co.grads, ao.grads, rows, taus=taus)
    torch.cuda.synchronize()
    np.testing.assert_allclose(cl.item(), z["n32/critic_loss"], rtol=bar["loss"])
    np.testing.assert_allclose(al.item(), z["n32/actor_loss"], rtol=bar["loss"])
    _check_params(loc.critic, z, "n32after/critic/", before["critic"], ops)
    _check_params(loc.actor, z, "n32after/actor/", before["actor"], ops)


@pytest.mark.parametrize("ops", ["f32", "bf16"])
def test_fused_iqn_matches_reference(ops):
    """Three train_IQN steps (max over actions per tau in the target, agent.py:451-452)."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_iqn import FusedIQNState, iqn_update_fused
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    z = np.load(eo.GOLDEN + "/learn_iqn.npz")
    ag = Agent(seed=100, agent_type="IQN")
    net = ag.policy_local
    for k, v in net.state_dict().items():
        np.testing.assert_array_equal(v.cpu().numpy(), z["init/" + k])
    opt = FusedAdam(net.parameters(), lr=1e-4, operands=ops)
    st = FusedIQNState(net, ag.policy_target, 64, 8, operands=ops)
    bar = BARS[ops]
    before = _snapshot(net)
    for step in range(3):
        rows = _rows(z, f"step{step}/", discrete=True)
        taus = torch.from_numpy(z[f"step{step}/taus"][..., 0]).cuda().contiguous()
        loss, gn = iqn_update_fused(st, net, opt, opt.grads, rows, taus=taus)
        torch.cuda.synchronize()
        np.testing.assert_allclose(loss.item(), z[f"step{step}/loss"], rtol=bar["loss"])
        np.testing.assert_allclose([gn.item()], z[f"step{step}/grad_norms"], rtol=bar["norm"])
        if step in (0, 2):
            _check_params(net, z, f"after{step}/", before, ops)


@pytest.mark.parametrize("ops", ["f32", "bf16"])
def test_fused_iqn_act_matches_reference(ops):
    """act_iqn (agent.py:227-256) on the captured state and K = 32 taus, greedy: the action kernel
    (mean over the 32 quantile samples, argmax) picks the reference's action."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_iqn import IqnPack, iqn_act
    z = np.load(eo.GOLDEN + "/learn_iqn.npz")
    ag = Agent(seed=100, agent_type="IQN")
    for k, v in ag.policy_local.state_dict().items():
        v.copy_(torch.tensor(z["after2/" + k]))
    pack = IqnPack(ag.policy_local, ops)
    obs = torch.zeros(1, 40, device="cuda")
    obs[0, 0:7] = torch.tensor(z["act/state_self"])
    objs = z["act/state_obj"]
    obs[0, 7:7 + 5 * len(objs)] = torch.tensor(objs.reshape(-1))
    obs[0, 32:32 + len(objs)] = 1.0
    acts = torch.zeros(1, 2, dtype=torch.float64, device="cuda")
    step = torch.zeros(1, dtype=torch.int64, device="cuda")
    taus = torch.from_numpy(z["act/taus"].reshape(32)).cuda()
    iqn_act(pack, None, acts, step, 1, 1e9, 0.25, 0.0, 0.0, 0, taus=taus, obs=obs)
    torch.cuda.synchronize()
    q = z["act/quantiles"][0].mean(0)
    best = int(acts[0, 0].item())
    if ops == "f32":
        assert best == int(z["act/action"])
    else:   # bf16: the chosen action's mean quantile within 1e-2 of the best
        assert q.max() - q[best] < 1e-2, (best, int(z["act/action"]), q.max() - q[best])


def test_fused_ac_iqn_bench_shape_bf16_tracks_f32():
    """The bench shape (B = 4096, N = N' = 32): one update of the bf16 training build against the
    f32 build of the same kernels on the same random batch and taus."""
    from distributional_rl_decision_and_control_amd.fused_update import ac_iqn_update_fused2
    B, N = 4096, 32
    g = torch.Generator(device="cuda").manual_seed(11)
    rows = torch.zeros(B, 88, device="cuda")
    for c in (0, 40):
        rows[:, c:c + 7] = torch.randn(B, 7, generator=g, device="cuda") * 3
        rows[:, c + 7:c + 32] = torch.randn(B, 25, generator=g, device="cuda") * 3
        rows[:, c + 32:c + 37] = (torch.rand(B, 5, generator=g, device="cuda") > 0.4).float()
    rows[:, 80:82] = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
    rows[:, 82] = torch.randn(B, generator=g, device="cuda")
    rows[:, 83] = (torch.rand(B, generator=g, device="cuda") > 0.9).float()
    taus = torch.rand(3, B, N, generator=g, device="cuda")
    out, deltas = {}, {}
    for ops in ("f32", "bf16"):
        loc, tgt, ao, co, st = _ac_iqn(ops, B, N)
        p0 = torch.cat([co.flat, ao.flat]).clone()
        res = ac_iqn_update_fused2(st, loc, ao, co, co.grads, ao.grads, rows, taus=taus)
        torch.cuda.synchronize()
        out[ops] = np.array([r.item() for r in res])
        deltas[ops] = (torch.cat([co.flat, ao.flat]) - p0).cpu().numpy()
    np.testing.assert_allclose(out["bf16"][:2], out["f32"][:2], rtol=2e-2)
    np.testing.assert_allclose(out["bf16"][2:], out["f32"][2:], rtol=5e-2)
    c = _cos(deltas["bf16"], deltas["f32"])
    print(f"bench shape: losses f32 {out['f32'][:2]}, bf16 {out['bf16'][:2]}; update cosine {c:.4f}")
    assert c > 0.95


def test_rollout_act_kernel_f32_matches_reference_actor():
    """The act kernel that produces every training action (actor_kernel<ACT>, asvrl_actor_forward MODE_ACT:
    Actor.forward, AC_IQN_model.py:284-323, + epsilon-greedy, agent.py:207-225) in the f32-operand build at
    epsilon = 0 against the reference's actor: the captured outputs of the seeded initial actor on
    no-object states (fwd/noobj_*), and the CPU restatement (oracle.learn_ref.actor_forward, f64) of the
    reference's actor with its initial and post-step-1 / post-step-3 weights on every F4 state (s and s').
    Bar: 1e-5 on actions. The bf16 build (the training path) at its stated 2 % of scale: test_fused_mlp_gpu."""
    from distributional_rl_decision_and_control_amd.fused_mlp import MlpPack, actor_act
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import AC_IQN_Policy
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    pol = AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1, 1], [-1, 1]], device="cuda", seed=100)

    def act(rows):
        pack = MlpPack(pol.actor, "actor", "f32")
        out = torch.empty(rows.shape[0], 2, dtype=torch.float64, device="cuda")
        step = torch.zeros(1, dtype=torch.int64, device="cuda")
        actor_act(pack, rows, out, step, 1, 1e6, 0.25, 0.0, 0.0, seed=3)   # epsilon 0 throughout
        torch.cuda.synchronize()
        return out.cpu().numpy()

    def load(prefix):
        with torch.no_grad():
            for k, v in pol.actor.state_dict().items():
                v.copy_(torch.tensor(z[prefix + "actor/" + k]))

    load("init/")
    ns = z["fwd/noobj_self"]
    rows = torch.zeros(ns.shape[0], 40, device="cuda")
    rows[:, 0:7] = torch.tensor(ns)
    np.testing.assert_allclose(act(rows), z["fwd/noobj_actions"], rtol=1e-5, atol=1e-6)
    states = []
    for st in ("step0/", "step1/", "step2/"):
        for p in ("s_", "ns_"):
            states.append((z[st + p + "self"], z[st + p + "obj"], z[st + p + "mask"]))
    S = np.concatenate([s[0] for s in states]), np.concatenate([s[1] for s in states]), \
        np.concatenate([s[2] for s in states])
    n = S[0].shape[0]
    rows = torch.zeros(n, 40, device="cuda")
    rows[:, 0:7] = torch.tensor(S[0])
    rows[:, 7:32] = torch.tensor(S[1]).reshape(n, 25)
    rows[:, 32:37] = torch.tensor(S[2])
    for prefix in ("init/", "after0/", "after2/"):
        load(prefix)
        w = {k: torch.tensor(z[prefix + "actor/" + k]).double() for k in pol.actor.state_dict()}
        ref = lr.actor_forward(w, tuple(torch.tensor(x).double() for x in S)).numpy()
        np.testing.assert_allclose(act(rows), ref, rtol=1e-5, atol=1e-6, err_msg=prefix)
