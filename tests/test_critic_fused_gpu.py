"""GPU: asvrl_critic_train_fused (forward + quantile-Huber + backward + trunk weight gradients in one
launch, asvrl_critic_fused.hip) against the two-kernel TRAIN path with its batched weight-gradient
launch over saved activations (asvrl_critic_train + asvrl_linear_wgrad_multi) -- the path the golden
tests pinned in round 1 -- on the same batch, taus and weights.

Bars: f32 build (libasvrl_f32.so): every critic gradient within 2e-5 of the tensor's scale (max |g|)
and the loss within 1e-6 rel. -- the two paths differ only in f32 summation order (bias added as the
MFMA's C input, per-workgroup row partials); bf16 build: per-tensor gradient cosine > 0.999 and norm
within 1 %, loss within 1e-4 rel. (the bf16 roundings of the activations are the same, the
accumulation orders are not; h2 enters the output layer's gradient as bf16). The fused launch is
deterministic (two runs bit-identical). The reference pin of the fused path itself is
test_learner_golden_gpu (train_AC_IQN at 1e-5 with the f32 build).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(B, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    rows = torch.zeros(B, 88, device="cuda")
    for c in (0, 40):
        rows[:, c:c + 7] = torch.randn(B, 7, generator=g, device="cuda") * 3
        rows[:, c + 7:c + 32] = torch.randn(B, 25, generator=g, device="cuda") * 3
        rows[:, c + 32:c + 37] = (torch.rand(B, 5, generator=g, device="cuda") > 0.4).float()
    rows[:, 80:82] = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
    rows[:, 82] = torch.randn(B, generator=g, device="cuda")
    rows[:, 83] = (torch.rand(B, generator=g, device="cuda") > 0.9).float()
    return rows, torch.rand(2, B, 0 + 1, generator=g, device="cuda")


def _critic_grads(ops, B, N, fused, rows, taus, seed=100, enc=False, tq=False, out=None):
    """The critic step's gradients (every critic .grad, reduced) and loss, without the optimizer.
    enc: the encoders' gradients formed inside the fused launch (parts.enc / parts.aenc) instead of
    the batched weight-gradient launch over dzF / dzG. tq: the target critic's forward inside the same
    launch (asvrl_critic_train_fused_tq) instead of asvrl_critic_forward (q_next poisoned with NaN
    before the launch); out["q_next"] receives the q_next the update read."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_critic import (TrainBuffers, critic_train, critic_train_fused,
                                                                          wout_groups)
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState, target_q
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    ag = Agent(seed=seed, agent_type="AC-IQN")
    loc, tgt = ag.policy_local, ag.policy_target
    FusedAdam(loc.actor.parameters(), lr=1e-4, operands=ops)
    co = FusedAdam(loc.critic.parameters(), lr=1e-4, operands=ops)
    st = FusedACIQNState(loc, tgt, B, N, operands=ops)
    critic, arena = loc.critic, st.arena
    bufs = None if fused else TrainBuffers(B, N, "cuda", ops)   # the two-kernel reference's activations
    s_rows, a_rows, r_col, d_col = rows[:, 0:40], rows[:, 80:82], rows[:, 82], rows[:, 83]
    co.grads.zero_()
    target_q(st, rows, taus[0], st.q_next, st.na)
    ae = critic.action_encoder[0]
    if tq:
        st.q_next.fill_(float("nan"))
        critic_train_fused(st.local_trunk, critic, taus[1], N, st.q_next.view(B, N), r_col, d_col, 0.99, s_rows,
                           a_rows, arena, tile_loss=st.tile_loss[0], encoders=True,
                           target=(st.target_trunk, taus[0], rows[:, 40:80], st.na))
    elif fused and enc:
        critic_train_fused(st.local_trunk, critic, taus[1], N, st.q_next.view(B, N), r_col, d_col, 0.99, s_rows,
                           a_rows, arena, tile_loss=st.tile_loss[0], encoders=True)
    elif fused:
        critic_train_fused(st.local_trunk, critic, taus[1], N, st.q_next.view(B, N), r_col, d_col, 0.99, s_rows,
                           a_rows, arena, dzF=st.dzF, dzG=st.dzG, xb=st.xb, tile_loss=st.tile_loss[0])
    else:
        tiles = wout_groups(B, N)
        wout = arena.take_tiles(tiles, 128)
        critic_train(st.local_trunk, None, None, taus[1], None, bufs, q_next=st.q_next.view(B, N), rewards=r_col,
                     dones=d_col, gamma=0.99, dzF=st.dzF, dzG=st.dzG, with_dFdG=False, tile_loss=st.tile_loss[0],
                     obs=s_rows, act=a_rows, xb=st.xb, wout_part=wout)
        arena.tiles(wout, tiles, critic.output_layer.weight.grad, critic.output_layer.bias.grad)
    with arena.batch():
        if enc:
            pass
        elif not fused:
            b = bufs
            arena.linear(b.dzc, b.cos, critic.cos_embedding.weight.grad, critic.cos_embedding.bias.grad)
            arena.linear(b.dz1, b.h0, critic.hidden_layer.weight.grad, critic.hidden_layer.bias.grad)
            arena.linear(b.dz2, b.h1g, critic.hidden_layer_2.weight.grad, critic.hidden_layer_2.bias.grad)
        if not enc:
            arena.fold(st.dzF, st.xb, critic)
            arena.small(st.dzG, a_rows, ae.weight.grad, ae.bias.grad)
    arena.scalar(st.tile_loss[0], st.losses[0:1])
    arena.flush()
    torch.cuda.synchronize()
    if out is not None:
        out["q_next"] = st.q_next.detach().cpu().numpy().copy()
    grads = {n: p.grad.detach().cpu().numpy().astype(np.float64).copy() for n, p in critic.named_parameters()}
    return grads, float(st.losses[0].item())


def _reference_grads(rows, taus, seed=100):
    """Critic gradients of the same step by torch autograd in f64 on the CPU (oracle/learn_ref.py's
    restatement of agent.py:395-414), from the same seeded initial weights."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    from oracle import learn_ref as lr
    ag = Agent(seed=seed, agent_type="AC-IQN")
    cw = {k: v.detach().cpu().double().requires_grad_(True) for k, v in ag.policy_local.critic.state_dict().items()}
    aw = {k: v.detach().cpu().double() for k, v in ag.policy_local.actor.state_dict().items()}
    x = rows.detach().cpu().double()
    B = x.shape[0]

    def st(c):
        return x[:, c:c + 7], x[:, c + 7:c + 32].reshape(B, 5, 5), x[:, c + 32:c + 37]
    t = taus.detach().cpu().double()
    N = t.shape[2]
    with torch.no_grad():
        na = lr.actor_forward(aw, st(40))
        qn = lr.critic_forward({k: v.detach() for k, v in cw.items()}, st(40), na, t[0].view(B, N, 1))
    qt = x[:, 82:83] + 0.99 * qn * (1.0 - x[:, 83:84])
    qe = lr.critic_forward(cw, st(0), x[:, 80:82], t[1].view(B, N, 1))
    loss = lr.quantile_huber(qt, qe, t[1].view(B, N, 1))
    names = list(cw)
    g = torch.autograd.grad(loss, [cw[n] for n in names])
    return {n: gi.numpy() for n, gi in zip(names, g)}, float(loss)


def _cos(x, y):
    x, y = x.reshape(-1), y.reshape(-1)
    return float(x @ y / (np.linalg.norm(x) * np.linalg.norm(y) + 1e-300))


@pytest.mark.parametrize("ops,B,N", [("f32", 64, 8), ("f32", 64, 16), ("f32", 64, 32), ("f32", 256, 32),
                                     ("bf16", 64, 8), ("bf16", 128, 16), ("bf16", 4096, 32),
                                     ("bf16", 608, 32)])   # 304 rounds over 256 workgroups: uneven
def test_fused_train_matches_two_kernel_path(ops, B, N):
    rows, _ = _batch(B, 5 + N)
    g = torch.Generator(device="cuda").manual_seed(7 + B)
    taus = torch.rand(2, B, N, generator=g, device="cuda")
    gf, lf = _critic_grads(ops, B, N, True, rows, taus)
    gu, lu = _critic_grads(ops, B, N, False, rows, taus)
    if ops == "f32" and B <= 256:
        # both paths against torch autograd in f64 (a wrong path shows as the one far from it)
        gr, lr_ = _reference_grads(rows, taus)
        for n in gr:
            scale = np.abs(gr[n]).max() + 1e-30
            ef, eu = np.abs(gf[n] - gr[n]).max() / scale, np.abs(gu[n] - gr[n]).max() / scale
            print(f"{n:28s} fused {ef:.2e}  two-kernel {eu:.2e}")
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


def test_fused_train_deterministic():
    B, N = 1024, 32
    rows, _ = _batch(B, 3)
    taus = torch.rand(2, B, N, generator=torch.Generator(device="cuda").manual_seed(4), device="cuda")
    g1, l1 = _critic_grads("bf16", B, N, True, rows, taus)
    g2, l2 = _critic_grads("bf16", B, N, True, rows, taus)
    assert l1 == l2
    for n in g1:
        np.testing.assert_array_equal(g1[n], g2[n], err_msg=n)


@pytest.mark.parametrize("ops,B,N", [("f32", 64, 8), ("f32", 64, 32), ("f32", 256, 16),
                                     ("bf16", 64, 8), ("bf16", 128, 16), ("bf16", 4096, 32)])
def test_fused_encoder_grads_in_kernel(ops, B, N):
    """parts.enc / parts.aenc (ABI 16): the observation encoders' gradients (folded over the five
    objects) and the action encoder's, summed inside the fused launch from its own dzF / dzG, against
    the batched weight-gradient launch over the dzF / dzG it writes out (and, f32 at small B, against
    f64 autograd). f32: 2e-5 of scale; bf16: cosine > 0.999, norm within 1 % (the out-of-kernel path
    rounds dzF and the inputs to bf16, the in-kernel one keeps them f32). Every other gradient and the
    loss are unchanged bit for bit; the launch stays deterministic."""
    from distributional_rl_decision_and_control_amd.fused_critic import fused_variant
    rows, _ = _batch(B, 11 + N)
    g = torch.Generator(device="cuda").manual_seed(17 + B)
    taus = torch.rand(2, B, N, generator=g, device="cuda")
    # the one-wave-per-SIMD kernel for both forms (the per-sample dzF / dzG form has no two-wave variant, and the
    # bit-identity below is between two forms of ONE kernel); variant 8: tests/test_critic_fused8_gpu.py
    with fused_variant(4, ops):
        ge, le = _critic_grads(ops, B, N, True, rows, taus, enc=True)
        gf, lf = _critic_grads(ops, B, N, True, rows, taus)
    assert le == lf
    enc_names = [n for n in gf if "encoder" in n]
    assert len(enc_names) == 6
    for n in gf:
        if n not in enc_names:
            np.testing.assert_array_equal(ge[n], gf[n], err_msg=n)
    if ops == "f32":
        ref = _reference_grads(rows, taus)[0] if B <= 256 else gf
        for n in enc_names:
            scale = np.abs(ref[n]).max() + 1e-30
            assert np.abs(ge[n] - ref[n]).max() / scale < 2e-5, n
    else:
        for n in enc_names:
            c = _cos(ge[n], gf[n])
            ratio = np.linalg.norm(ge[n]) / np.linalg.norm(gf[n])
            assert c > 0.999 and abs(ratio - 1) < 1e-2, (n, c, ratio)
    with fused_variant(4, ops):
        g2, _ = _critic_grads(ops, B, N, True, rows, taus, enc=True)
    for n in enc_names:
        np.testing.assert_array_equal(ge[n], g2[n], err_msg=n)


@pytest.mark.parametrize("ops,B,N", [("f32", 64, 8), ("f32", 64, 32), ("f32", 256, 16),
                                     ("bf16", 64, 8), ("bf16", 128, 16), ("bf16", 608, 32), ("bf16", 4096, 32)])
def test_fused_train_with_target_critic_in_launch(ops, B, N):
    """asvrl_critic_train_fused_tq (ABI 20), kernel variant 4: each workgroup computes q_next = target_critic(s', a', tau') for
    the samples its rounds update (asvrl_critic.hip's FWD tile, compiled into the fused launch ahead of the
    contraction pragma), then runs the update. Against asvrl_critic_forward followed by the plain fused launch:
    q_next bit-identical (every sample: 608 x 32 gives 304 rounds over 256 workgroups, uneven), and so every
    gradient and the loss bit-identical too."""
    from distributional_rl_decision_and_control_amd.fused_critic import fused_variant
    rows, _ = _batch(B, 21 + N)
    g = torch.Generator(device="cuda").manual_seed(27 + B)
    taus = torch.rand(2, B, N, generator=g, device="cuda")
    o1, o2 = {}, {}
    with fused_variant(4, ops):   # this kernel's target pass is asvrl_critic_forward's tile (variant 8: test_critic_fused8_gpu)
        g1, l1 = _critic_grads(ops, B, N, True, rows, taus, enc=True, out=o1)
        g2, l2 = _critic_grads(ops, B, N, True, rows, taus, enc=True, tq=True, out=o2)
    assert np.isfinite(o2["q_next"]).all()
    np.testing.assert_array_equal(o2["q_next"], o1["q_next"])
    assert l1 == l2
    for n in g1:
        np.testing.assert_array_equal(g2[n], g1[n], err_msg=n)
