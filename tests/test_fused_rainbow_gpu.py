"""GPU: Rainbow's hand-written kernels (asvrl_rainbow.hip, fused_rainbow.py) against the torch fp32
restatement of Rainbow_Policy / train_Rainbow (policy/Rainbow_model.py, learner.rainbow_update,
itself pinned to the reference's train_Rainbow by tests/test_agent_gpu.py).

Bars: composed noisy weights bit-exact (mu + sigma * eps, same f32 ops); factorised reset noise is
rank-1 with the moments of f(N(0,1)). The network kernel (asvrl_rainbow_net.hip) in the f32 build:
greedy act identical to the torch argmax on >= 99.5% of rows (the rest within 1e-5 of the best
expected value: float near-ties), p(s', a*) within 1e-5; one fused update vs rainbow_update with the
same target noise: per-sample loss 1e-4, gradient norm 1e-4, parameters 1e-5. The bf16 build (the
training path): act within 5e-3 of the best expected value on every row, p(s', a*) within 2e-3, the
update's per-sample loss within 2 % and gradient cosine > 0.99 of the f32 reference update."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _nets(seed=9):
    from distributional_rl_decision_and_control_amd.policy.Rainbow_model import Rainbow_Policy
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    local = Rainbow_Policy(**DEFAULT_NET, action_size=25, atoms=51, device="cuda", seed=seed).to("cuda")
    target = copy.deepcopy(local)
    for p in target.parameters():
        p.requires_grad_(False)
    return local, target


def _rows(B, seed=1):
    g = torch.Generator(device="cuda").manual_seed(seed)
    rows = torch.zeros(B, 88, device="cuda")
    rows[:, 0:37] = torch.randn(B, 37, device="cuda", generator=g)
    rows[:, 40:77] = torch.randn(B, 37, device="cuda", generator=g)
    rows[:, 32:37] = (rows[:, 32:37] > 0).float()
    rows[:, 72:77] = (rows[:, 72:77] > 0).float()
    rows[:, 80] = torch.randint(0, 25, (B,), device="cuda", generator=g).float()
    rows[:, 82] = torch.randn(B, device="cuda", generator=g)
    rows[:, 83] = (torch.rand(B, device="cuda", generator=g) > 0.2).float()
    rows[:, 84] = torch.rand(B, device="cuda", generator=g) * 0.9 + 0.1
    return rows


def test_noisy_compose_and_reset():
    from distributional_rl_decision_and_control_amd.fused_rainbow import NOISY, NoisyPack
    local, target = _nets()
    pack = NoisyPack(local)
    pack.compose()
    W, _ = pack.weights()
    for n in NOISY:
        L = getattr(local, n)
        torch.testing.assert_close(W[n][0], L.weight_mu + L.weight_sigma * L.weight_epsilon, rtol=0, atol=0)
        torch.testing.assert_close(W[n][1], L.bias_mu + L.bias_sigma * L.bias_epsilon, rtol=0, atol=0)
    tp = NoisyPack(target)
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    tp.reset(7, ctr)
    Wt, _ = tp.weights()
    fx = []
    for n in NOISY:
        L = getattr(target, n)
        ew, eb = L.weight_epsilon, L.bias_epsilon
        # eps_w = f(eps_out) f(eps_in)^T with f(eps_out) = eps_b: rank 1
        ein = ew[0] / eb[0]
        torch.testing.assert_close(ew, torch.outer(eb, ein), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(Wt[n][0], L.weight_mu + L.weight_sigma * ew, rtol=0, atol=0)
        fx.append(eb.cpu().numpy())
    fx = np.concatenate(fx)
    assert abs(fx.mean()) < 0.05 and abs((fx ** 2).mean() - np.sqrt(2 / np.pi)) < 0.05
    ctr += 1
    tp.reset(7, ctr)
    assert not torch.equal(target.output_layer_a.bias_epsilon.cpu(), torch.from_numpy(fx[-1275:]))


@pytest.mark.parametrize("ops", ["f32", "bf16"])
def test_act_greedy_matches_torch(ops):
    from distributional_rl_decision_and_control_amd.fused_rainbow import FusedRainbow
    local, target = _nets()
    sup = torch.linspace(-1.0, 1.0, 51, device="cuda")
    fr = FusedRainbow(local, target, 64, sup, operands=ops)
    N = 4096
    obs = _rows(N)[:, 0:40].contiguous()
    acts = torch.zeros(N, 2, dtype=torch.float64, device="cuda")
    step = torch.zeros(1, dtype=torch.int64, device="cuda")
    # eps schedule pinned at 0 (initial = final = 0): greedy
    fr.act(obs, acts, step, 1, 1e9, 0.25, 0.0, 0.0, 3)
    with torch.no_grad():
        local.train()
        p = local((obs[:, 0:7], obs[:, 7:32].reshape(N, 5, 5), obs[:, 32:37]))
        Q = (p * sup).sum(2)
    ref = Q.argmax(1)
    got = acts[:, 0].long()
    same = (got == ref).float().mean().item()
    gap = (Q.max(1).values - Q.gather(1, got[:, None])[:, 0]).abs().max().item()
    print(f"{ops}: argmax agreement {same:.4f}, max expected-value gap {gap:.2e}")
    if ops == "f32":
        assert same >= 0.995 and gap < 1e-5
    else:
        assert same >= 0.9 and gap < 5e-3
    # eps = 1: uniform exploration over the 25 actions
    fr.act(obs, acts, step, 1, 1e9, 0.25, 1.0, 1.0, 3)
    h = np.bincount(acts[:, 0].long().cpu().numpy(), minlength=25)
    assert h.min() > 0.5 * N / 25


@pytest.mark.parametrize("ops", ["f32", "bf16"])
def test_target_pick_matches_torch(ops):
    """The double-Q argmax (online net, s') and p(s', a*) of the target net (agent.py:605-612)."""
    from distributional_rl_decision_and_control_amd.fused_rainbow import FusedRainbow
    local, target = _nets()
    sup = torch.linspace(-1.0, 1.0, 51, device="cuda")
    N = 2048 + 17   # a ragged last tile
    fr = FusedRainbow(local, target, N, sup, operands=ops)
    ns = _rows(N, 5)[:, 40:80]
    a_star = torch.zeros(N, dtype=torch.int64, device="cuda")
    p_star = torch.zeros(N, 51, device="cuda")
    fr.img.run("asvrl_rainbow_net_argmax", fr.img.io(ns, fr.support, act_idx=a_star.data_ptr()))
    fr.timg.run("asvrl_rainbow_net_pick", fr.timg.io(ns, fr.support, act_idx=a_star.data_ptr(), p_out=p_star.data_ptr()))
    x = (ns[:, 0:7], ns[:, 7:32].reshape(N, 5, 5), ns[:, 32:37])
    with torch.no_grad():
        local.train()
        target.train()
        Q = (local(x) * sup).sum(2)
        pt = target(x)
    gap = (Q.max(1).values - Q.gather(1, a_star[:, None])[:, 0]).abs().max().item()
    ref_p = pt[torch.arange(N, device="cuda"), a_star]
    err = (p_star - ref_p).abs().max().item()
    print(f"{ops}: argmax agreement {(Q.argmax(1) == a_star).float().mean().item():.4f}, gap {gap:.2e}, p err {err:.2e}")
    if ops == "f32":
        assert gap < 1e-5 and err < 1e-5
    else:
        assert gap < 5e-3 and err < 2e-3


@pytest.mark.parametrize("B", [1024, 8192])  # 8192: split-K weight gradients (SPLITK_MIN_ROWS)
def test_fused_update_matches_rainbow_update(B):
    from distributional_rl_decision_and_control_amd.fused_rainbow import FusedRainbow
    from distributional_rl_decision_and_control_amd.learn_ops import split_rows
    from distributional_rl_decision_and_control_amd.learner import FlatGrads, rainbow_update
    rows = _rows(B)
    sup = torch.linspace(-1.0, 1.0, 51, device="cuda")
    local, target = _nets()
    ref_local, ref_target = copy.deepcopy(local), copy.deepcopy(target)
    grads = FlatGrads(local.parameters())
    opt = torch.optim.Adam(local.parameters(), lr=1e-4)
    fr = FusedRainbow(local, target, B, sup, operands="f32")
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    loss, gn = fr.update(opt, grads, rows, seed=11, counter_dev=ctr)
    # the reference update with the target noise the fused reset drew
    for a, b in zip(ref_target.buffers(), target.buffers()):
        a.copy_(b)
    rgrads = FlatGrads(ref_local.parameters())
    ropt = torch.optim.Adam(ref_local.parameters(), lr=1e-4)
    s, a, R, ns, nt = split_rows(rows)
    rloss, rgn = rainbow_update(ref_local, ref_target, ropt, rgrads, sup, s, a[:, 0].long(), R, ns, nt, rows[:, 84],
                                reset_target_noise=False)
    torch.testing.assert_close(loss, rloss, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gn, rgn, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(grads.flat, rgrads.flat, rtol=1e-3, atol=1e-6)
    for p, q in zip(local.parameters(), ref_local.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_fused_update_bf16_tracks_rainbow_update():
    from distributional_rl_decision_and_control_amd.fused_rainbow import FusedRainbow
    from distributional_rl_decision_and_control_amd.learn_ops import split_rows
    from distributional_rl_decision_and_control_amd.learner import FlatGrads, rainbow_update
    B = 8192
    rows = _rows(B)
    sup = torch.linspace(-1.0, 1.0, 51, device="cuda")
    local, target = _nets()
    ref_local, ref_target = copy.deepcopy(local), copy.deepcopy(target)
    grads = FlatGrads(local.parameters())
    fr = FusedRainbow(local, target, B, sup, operands="bf16")
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    loss, gn = fr.update(torch.optim.Adam(local.parameters(), lr=1e-4), grads, rows, seed=11, counter_dev=ctr)
    for a, b in zip(ref_target.buffers(), target.buffers()):
        a.copy_(b)
    rgrads = FlatGrads(ref_local.parameters())
    s, a, R, ns, nt = split_rows(rows)
    rloss, rgn = rainbow_update(ref_local, ref_target, torch.optim.Adam(ref_local.parameters(), lr=1e-4), rgrads, sup,
                                s, a[:, 0].long(), R, ns, nt, rows[:, 84], reset_target_noise=False)
    rel = ((loss - rloss).abs() / rloss.abs().clamp_min(1e-6)).max().item()
    g, rg = grads.flat.double(), rgrads.flat.double()
    cos = float(g @ rg / (g.norm() * rg.norm()))
    print(f"bf16 update: max per-sample loss rel {rel:.2e}, grad cosine {cos:.6f}")
    assert rel < 2e-2 and cos > 0.99
