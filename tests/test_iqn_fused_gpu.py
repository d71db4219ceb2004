"""GPU: asvrl_iqn_train_fused (train_IQN's local pass, agent.py:455-468 -- forward, gather at the taken
action, quantile-Huber, backward -- plus the weight gradients of the trunk and the 128 -> A output layer
in one launch, asvrl_critic_fused.hip on IQN_Policy's trunk) against the two-kernel path with its batched
weight-gradient launch over saved activations (asvrl_iqn_train + asvrl_linear_wgrad_multi), on the same
batch, taus and weights; the f32 build also against torch autograd on the CPU in f32, the reference's
own arithmetic (oracle/learn_ref.py; in f64 a cos-layer pre-activation within f32 rounding of 0 takes
the other side of the ReLU for one row at B = 256, for both GPU paths alike).

Bars as tests/test_critic_fused_gpu.py: f32 build every gradient within 2e-5 of the tensor's scale,
loss 1e-6 rel.; bf16 build gradient cosine > 0.999, norm within 1 %, loss 1e-4 rel. The reference pin
of the fused path through Agent.train is test_learner_golden_gpu.test_fused_iqn_matches_reference.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

A = 25


def _batch(B, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    rows = torch.zeros(B, 88, device="cuda")
    for c in (0, 40):
        rows[:, c:c + 7] = torch.randn(B, 7, generator=g, device="cuda") * 3
        rows[:, c + 7:c + 32] = torch.randn(B, 25, generator=g, device="cuda") * 3
        rows[:, c + 32:c + 37] = (torch.rand(B, 5, generator=g, device="cuda") > 0.4).float()
    rows[:, 80] = torch.randint(0, A, (B,), generator=g, device="cuda").float()
    rows[:, 82] = torch.randn(B, generator=g, device="cuda")
    rows[:, 83] = (torch.rand(B, generator=g, device="cuda") > 0.9).float()
    return rows


def _iqn_grads(ops, B, N, fused, rows, taus, seed=100, enc=True):
    """Every IQN_Policy .grad (reduced) and the loss of one train_IQN step, without the optimizer.
    enc: the fused launch forms the encoders' gradients itself (ABI 16) instead of the batched
    weight-gradient launch over its dzF."""
    from distributional_rl_decision_and_control_amd import fused_iqn as fi
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    ag = Agent(seed=seed, agent_type="IQN")
    net = ag.policy_local
    opt = FusedAdam(net.parameters(), lr=1e-4, operands=ops)
    st = fi.FusedIQNState(net, ag.policy_target, B, N, operands=ops)
    opt.grads.zero_()
    old, fi.FUSED_TRAIN = fi.FUSED_TRAIN, fused
    old_enc, fi.ENC_IN_KERNEL = fi.ENC_IN_KERNEL, enc
    try:
        fi.iqn_grads(st, net, rows, taus, 0.99, flush=True)
    finally:
        fi.FUSED_TRAIN, fi.ENC_IN_KERNEL = old, old_enc
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu().numpy().astype(np.float64).copy() for n, p in net.named_parameters()}
    return grads, float(st.loss[0].item())


def _reference_grads(rows, taus, seed=100):
    """The same step by torch autograd in f32 on the CPU (oracle/learn_ref.py's IQN forward and
    quantile-Huber loss, agent.py:449-468)."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    from oracle import learn_ref as lr
    ag = Agent(seed=seed, agent_type="IQN")
    cw = {k: v.detach().cpu().float().requires_grad_(True) for k, v in ag.policy_local.state_dict().items()}
    tw = {k: v.detach().cpu().float() for k, v in ag.policy_target.state_dict().items()}
    x = rows.detach().cpu().float()
    B = x.shape[0]

    def st(c):
        return x[:, c:c + 7], x[:, c + 7:c + 32].reshape(B, 5, 5), x[:, c + 32:c + 37]
    t = taus.detach().cpu().float()
    N = t.shape[2]
    with torch.no_grad():
        qn = lr.iqn_forward(tw, st(40), t[0].view(B, N, 1)).max(2)[0]
    qt = x[:, 82:83] + 0.99 * qn * (1.0 - x[:, 83:84])
    a = x[:, 80].long().view(B, 1, 1).expand(B, N, 1)
    qe = lr.iqn_forward(cw, st(0), t[1].view(B, N, 1)).gather(2, a).squeeze(2)
    loss = lr.quantile_huber(qt, qe, t[1].view(B, N, 1))
    names = list(cw)
    g = torch.autograd.grad(loss, [cw[n] for n in names])
    return {n: gi.double().numpy() for n, gi in zip(names, g)}, float(loss.detach())


def _cos(x, y):
    x, y = x.reshape(-1), y.reshape(-1)
    return float(x @ y / (np.linalg.norm(x) * np.linalg.norm(y) + 1e-300))


@pytest.mark.parametrize("ops,B,N", [("f32", 64, 8), ("f32", 64, 16), ("f32", 64, 32), ("f32", 256, 32),
                                     ("bf16", 64, 8), ("bf16", 128, 16), ("bf16", 4096, 32)])
def test_iqn_fused_train_matches_two_kernel_path(ops, B, N):
    rows = _batch(B, 11 + N)
    taus = torch.rand(2, B, N, generator=torch.Generator(device="cuda").manual_seed(3 + B), device="cuda")
    gf, lf = _iqn_grads(ops, B, N, True, rows, taus)
    gu, lu = _iqn_grads(ops, B, N, False, rows, taus)
    if ops == "f32" and B <= 256:
        gr, lr_ = _reference_grads(rows, taus)
        for n in gr:
            scale = np.abs(gr[n]).max() + 1e-30
            print(f"{n:28s} fused {np.abs(gf[n] - gr[n]).max() / scale:.2e}  "
                  f"two-kernel {np.abs(gu[n] - gr[n]).max() / scale:.2e}")
        for n in gr:
            scale = np.abs(gr[n]).max() + 1e-30
            assert np.abs(gf[n] - gr[n]).max() / scale < 2e-5, n
        np.testing.assert_allclose(lf, lr_, rtol=1e-5)
    if ops == "f32":
        np.testing.assert_allclose(lf, lu, rtol=1e-6)
        for n in gu:
            scale = np.abs(gu[n]).max() + 1e-30
            err = np.abs(gf[n] - gu[n]).max() / scale
            assert err < 2e-5, (n, err)
    else:
        np.testing.assert_allclose(lf, lu, rtol=1e-4)
        for n in gu:
            if np.abs(gu[n]).max() == 0:
                continue
            c = _cos(gf[n], gu[n])
            ratio = np.linalg.norm(gf[n]) / np.linalg.norm(gu[n])
            assert c > 0.999 and abs(ratio - 1) < 1e-2, (n, c, ratio)


def test_iqn_fused_train_deterministic():
    B, N = 1024, 32
    rows = _batch(B, 5)
    taus = torch.rand(2, B, N, generator=torch.Generator(device="cuda").manual_seed(6), device="cuda")
    g1, l1 = _iqn_grads("bf16", B, N, True, rows, taus)
    g2, l2 = _iqn_grads("bf16", B, N, True, rows, taus)
    assert l1 == l2
    for n in g1:
        np.testing.assert_array_equal(g1[n], g2[n], err_msg=n)


@pytest.mark.parametrize("ops,B,N", [("f32", 64, 8), ("f32", 256, 32), ("bf16", 64, 8), ("bf16", 4096, 32)])
def test_iqn_fused_encoder_grads_in_kernel(ops, B, N):
    """parts.enc (ABI 16) on IQN_Policy: the observation encoders' gradients summed in the fused launch
    (register accumulators; no LDS to spare at N = 8) against the batched launch over its dzF. Every
    other gradient and the loss bit-identical; encoders f32 2e-5 of scale, bf16 cosine > 0.999."""
    rows = _batch(B, 21 + N)
    taus = torch.rand(2, B, N, generator=torch.Generator(device="cuda").manual_seed(9 + B), device="cuda")
    ge, le = _iqn_grads(ops, B, N, True, rows, taus, enc=True)
    gf, lf = _iqn_grads(ops, B, N, True, rows, taus, enc=False)
    assert le == lf
    enc_names = [n for n in gf if "encoder" in n]
    assert len(enc_names) == 4
    for n in gf:
        if n not in enc_names:
            np.testing.assert_array_equal(ge[n], gf[n], err_msg=n)
    for n in enc_names:
        if ops == "f32":
            scale = np.abs(gf[n]).max() + 1e-30
            assert np.abs(ge[n] - gf[n]).max() / scale < 2e-5, n
        else:
            c = _cos(ge[n], gf[n])
            ratio = np.linalg.norm(ge[n]) / np.linalg.norm(gf[n])
            assert c > 0.999 and abs(ratio - 1) < 1e-2, (n, c, ratio)


@pytest.mark.parametrize("ops,B,N", [("bf16", 64, 8), ("bf16", 64, 16), ("bf16", 256, 32), ("bf16", 4096, 32),
                                     ("f32", 64, 8), ("f32", 256, 32)])
def test_iqn_target_max_in_launch_matches_separate(ops, B, N):
    """asvrl_iqn_train_fused_tq (ABI 24): the target network's max over the actions (agent.py:451-452) computed
    inside the fused launch, each workgroup for the samples it updates, against asvrl_iqn_forward_max + the
    fused launch: the same tile code on the same inputs, so q_next, every gradient and the loss are bit-identical
    (q_next poisoned with NaN before the launch that must write it)."""
    from distributional_rl_decision_and_control_amd import fused_iqn as fi
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    rows = _batch(B, 77)
    taus = torch.rand(2, B, N, generator=torch.Generator(device="cuda").manual_seed(78), device="cuda")
    out = {}
    for tq in (False, True):
        ag = Agent(seed=100, agent_type="IQN")
        net = ag.policy_local
        with torch.no_grad():   # a target network different from the local one
            for p in ag.policy_target.parameters():
                p.add_(0.05 * p.abs().mean() * torch.randn(p.shape, generator=torch.Generator().manual_seed(5)).to(p.device))
        opt = FusedAdam(net.parameters(), lr=1e-4, operands=ops)
        st = fi.FusedIQNState(net, ag.policy_target, B, N, operands=ops, target_in_fused=tq)
        opt.grads.zero_()
        st.q_next.fill_(float("nan"))
        if tq and ops == "f32":   # the learner keeps the separate launch in the f32 build: call the entry itself
            fi.iqn_train_fused(st.local, net, taus[1], N, st.q_next.view(B, N), rows[:, 80], rows[:, 82], rows[:, 83],
                               0.99, rows[:, 0:40], st.arena, tile_loss=st.tile_loss, encoders=True,
                               target=(st.target, taus[0], rows[:, 40:80]))
            st.arena.scalar(st.tile_loss, st.loss)
            st.arena.flush()
        else:
            fi.iqn_grads(st, net, rows, taus, 0.99, flush=True)
        torch.cuda.synchronize()
        out[tq] = ({n: p.grad.detach().clone() for n, p in net.named_parameters()}, st.loss.clone(), st.q_next.clone())
    (ga, la, qa), (gb, lb, qb) = out[False], out[True]
    assert torch.isfinite(qa).all() and torch.equal(qa, qb), float((qa - qb).abs().nan_to_num(1e30).max())
    assert torch.equal(la, lb), (la, lb)
    for n in ga:
        assert torch.equal(ga[n], gb[n]), (n, float((ga[n] - gb[n]).abs().max()))
