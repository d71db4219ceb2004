"""GPU parity of the learner kernels.

  * C51 projection vs the reference's own target distribution m captured from
    Agent.train_Rainbow (agent.py:616-631): bit-exact, plus the C oracle at B = 65536.
  * Quantile-Huber loss/gradient vs a plain torch fp32 autograd restatement of
    agent.py:406-412 + calculate_huber_loss (agent.py:701-707): rtol 1e-5.
  * Replay ring push/sample vs a host model of ReplayBuffer.add/sample order.
"""
import numpy as np
import pytest
import torch

from oracle import env_oracle as eo

pytestmark = pytest.mark.gpu


def _c51(pns_a, R, nt, support, gamma_n=0.99 ** 3):
    from distributional_rl_decision_and_control_amd import learn_ops
    return learn_ops.c51_project(pns_a, R, nt, support, vmin=-1.0, vmax=1.0, gamma_n=gamma_n)


@pytest.mark.parametrize("tag", ["b64", "b1024"])
def test_c51_bit_exact_vs_reference(tag):
    z = np.load(eo.GOLDEN + "/learn_rainbow.npz")
    dev = "cuda"
    m = _c51(torch.from_numpy(z[tag + "/pns_a"]).to(dev), torch.from_numpy(z[tag + "/returns"]).to(dev),
             torch.from_numpy(z[tag + "/nonterminal"]).to(dev).reshape(-1),
             torch.from_numpy(z[tag + "/support"]).to(dev))
    np.testing.assert_array_equal(m.cpu().numpy(), z[tag + "/m"])


def test_c51_large_batch_vs_oracle():
    rs = np.random.RandomState(0)
    B = 65536
    p = rs.dirichlet(np.ones(51), size=B).astype(np.float32)
    R = rs.uniform(-2, 2, size=B).astype(np.float32)
    R[::97] = np.round(R[::97] * 25) / 25  # on-grid returns (l == u cases)
    nt = rs.randint(0, 2, size=B).astype(np.float32)
    sup = torch.linspace(-1.0, 1.0, 51).numpy()
    ref = eo.c51_project(p, R, nt, sup)
    got = _c51(torch.from_numpy(p).cuda(), torch.from_numpy(R).cuda(), torch.from_numpy(nt).cuda(),
               torch.from_numpy(sup).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_allclose(got.sum(1), p.sum(1), rtol=1e-5)


def _qh_torch(qt, qe, tau, kappa=1.0):
    """agent.py:401-412 in torch fp32 (qt: (B,Np) targets, qe: (B,N) expected, tau: (B,N))."""
    Q_targets = qt.unsqueeze(1)            # (B, 1, Np)
    Q_expected = qe.unsqueeze(-1)          # (B, N, 1)
    td = Q_targets - Q_expected            # (B, N, Np)
    huber = torch.where(td.abs() <= kappa, 0.5 * td.pow(2), kappa * (td.abs() - 0.5 * kappa))
    ql = abs(tau.unsqueeze(-1) - (td.detach() < 0).float()) * huber / kappa
    return ql.sum(dim=1).mean(dim=1).mean()


@pytest.mark.parametrize("B,N,Np", [(64, 8, 8), (64, 32, 32), (4096, 32, 32), (7, 65, 3)])
def test_quantile_huber_vs_torch(B, N, Np):
    from distributional_rl_decision_and_control_amd import learn_ops
    g = torch.Generator().manual_seed(B + N)
    qt = (torch.randn(B, Np, generator=g) * 2).cuda()
    qe = (torch.randn(B, N, generator=g) * 2).requires_grad_(False).cuda()
    tau = torch.rand(B, N, generator=g).cuda()
    qe_ref = qe.clone().requires_grad_(True)
    ref = _qh_torch(qt, qe_ref, tau)
    ref.backward()
    qe_k = qe.clone().requires_grad_(True)
    loss = learn_ops.quantile_huber_loss(qt, qe_k, tau, 1.0)
    loss.backward()
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(qe_k.grad, qe_ref.grad, rtol=1e-5, atol=1e-7)


def test_replay_push_and_sample():
    from distributional_rl_decision_and_control_amd import learn_ops
    from distributional_rl_decision_and_control_amd._abi import OBS_DIM, TR_DIM
    rs = np.random.RandomState(1)
    n, cap = 1000, 2500
    ring = learn_ops.DeviceReplay(cap, device="cuda")
    host_rows = []
    for it in range(4):
        obs_prev = torch.from_numpy(rs.randn(n, OBS_DIM).astype(np.float32)).cuda()
        obs_next = torch.from_numpy(rs.randn(n, OBS_DIM).astype(np.float32)).cuda()
        cnt = torch.from_numpy(rs.randint(-1, 6, size=n).astype(np.int8)).cuda()
        act = torch.from_numpy(rs.randn(n, 2)).cuda()
        rew = torch.from_numpy(rs.randn(n)).cuda()
        done = torch.from_numpy(rs.randint(0, 2, size=n).astype(np.uint8)).cuda()
        ring.push(obs_prev, obs_next, cnt, act, rew, done)
        c = cnt.cpu().numpy()
        for k in np.nonzero(c >= 0)[0]:
            row = np.zeros(TR_DIM, np.float32)
            row[:OBS_DIM] = obs_prev[k].cpu().numpy()
            row[OBS_DIM:2 * OBS_DIM] = obs_next[k].cpu().numpy()
            row[80], row[81] = np.float32(act[k, 0].item()), np.float32(act[k, 1].item())
            row[82] = np.float32(rew[k].item())
            row[83] = float(done[k].item())
            host_rows.append(row)
    host_rows = host_rows[-cap:]  # deque(maxlen=cap) semantics
    assert ring.size() == len(host_rows)
    idx = rs.choice(len(host_rows), 64, replace=False)
    got = ring.gather(torch.from_numpy(idx.astype(np.int64)).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, np.stack([host_rows[i] for i in idx]))
    s1 = ring.sample(256, seed=5, counter=9).cpu().numpy()
    s2 = ring.sample(256, seed=5, counter=9).cpu().numpy()
    np.testing.assert_array_equal(s1, s2)
    hs = {r.tobytes() for r in host_rows}
    assert all(r.tobytes() in hs for r in s1)
