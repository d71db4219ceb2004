"""CPU: the bf16-build restatement of the critic step (oracle/learn_ref.critic_step_bf16) pinned before it is
trusted as the checker of the benched kernel (tests/test_critic_bf16_oracle_gpu.py).

With its rounding switched off it must be the reference's critic step: on the reference's own N = 32 batch
(tests/golden/learn_ac_iqn.npz, captured from agent.py:386-432) its loss equals the captured critic loss,
its gradient norm the captured pre-clip norm, and every gradient torch autograd of the fixture-pinned f64
restatement (oracle/learn_ref.critic_forward + quantile_huber). With bf16 rounding on it stays within the
bf16 build's stated bars of the same numbers (the rounding points move the loss by < 2 %)."""
import numpy as np
import torch

from oracle import env_oracle as eo
from oracle import learn_ref as lr


def _case():
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    p = "n32/"
    B = z[p + "s_self"].shape[0]
    d64 = lambda k: torch.tensor(z[k], dtype=torch.float64)   # noqa: E731
    s = (d64(p + "s_self"), d64(p + "s_obj").reshape(B, 5, 5), d64(p + "s_mask"))
    ns = (d64(p + "ns_self"), d64(p + "ns_obj").reshape(B, 5, 5), d64(p + "ns_mask"))
    cw = {k[len("init/critic/"):]: d64(k) for k in z.keys() if k.startswith("init/critic/")}
    aw = {k[len("init/actor/"):]: d64(k) for k in z.keys() if k.startswith("init/actor/")}
    taus = d64(p + "taus")   # (3, B, N, 1)
    with torch.no_grad():   # the target networks are the initial ones (TAU = 1 copies)
        qn = lr.critic_forward(cw, ns, lr.actor_forward(aw, ns), taus[0])
    return z, p, s, d64(p + "a"), d64(p + "r"), d64(p + "d"), taus, cw, qn


def test_bf16_restatement_without_rounding_is_the_reference_critic_step():
    z, p, s, a, r, d, taus, cw, qn = _case()
    B, N = taus.shape[1], taus.shape[2]
    loss, g = lr.critic_step_bf16(cw, s, a, qn, r, d, taus[1, ..., 0], rnd=lambda t: t)
    np.testing.assert_allclose(loss, float(z[p + "critic_loss"]), rtol=1e-5)
    gn = float(torch.sqrt(sum((x * x).sum() for x in g.values())))
    np.testing.assert_allclose(gn, float(z[p + "grad_norms"][0]), rtol=1e-4)
    # torch autograd of the fixture-pinned restatement, f64
    w = {k: v.clone().requires_grad_(True) for k, v in cw.items()}
    qt = r.view(B, 1) + 0.99 * qn * (1.0 - d.view(B, 1))
    ref_loss = lr.quantile_huber(qt, lr.critic_forward(w, s, a, taus[1]), taus[1])
    names = list(w)
    ref = dict(zip(names, torch.autograd.grad(ref_loss, [w[n] for n in names])))
    assert abs(loss - float(ref_loss.detach())) < 1e-12 * max(1.0, abs(loss))
    for n in names:
        np.testing.assert_allclose(g[n].numpy(), ref[n].numpy(), rtol=1e-9, atol=1e-12 * float(ref[n].abs().max()),
                                   err_msg=n)


def test_bf16_restatement_stays_within_the_bf16_bars():
    z, p, s, a, r, d, taus, cw, qn = _case()
    loss, g = lr.critic_step_bf16(cw, s, a, qn, r, d, taus[1, ..., 0])
    np.testing.assert_allclose(loss, float(z[p + "critic_loss"]), rtol=2e-2)
    gn = float(torch.sqrt(sum((x * x).sum() for x in g.values())))
    np.testing.assert_allclose(gn, float(z[p + "grad_norms"][0]), rtol=5e-2)
    l0, g0 = lr.critic_step_bf16(cw, s, a, qn, r, d, taus[1, ..., 0], rnd=lambda t: t)
    assert loss != l0   # the rounding points are live
