"""GPU: the EXACT launch the bench times -- asvrl_critic_train_fused_tq in the bf16 training build (libasvrl.so),
N = 32 with stage-ahead, the encoders' gradients formed in the launch (ENC_IN_KERNEL) and the TARGET critic's
forward inside the same launch (TARGET_IN_FUSED) -- against the bf16-build restatement of the critic step
(oracle/learn_ref.critic_step_bf16, pinned on CPU by tests/test_bf16_oracle_cpu.py), which rounds to bf16 exactly
where the kernel does and accumulates in f64. The separate-launch form (asvrl_critic_train_fused, the f32 parity
build's and the DP path's launch) is checked the same way.

The target quantiles are the ORACLE's: q_next = learn_ref.critic_forward_bf16(target critic, s', a', tau') -- the
target forward's own rounding points -- from the next states, the next actions the launch read (the target actor's
output, an earlier launch) and the launch's taus. The launch's in-kernel q_next is checked against it (within
Q_L2 relative over the tensor, any row within Q_MAX of the scale), and the gradients are compared against the restatement fed the oracle's q_next, so the
in-launch target pass is oracle-checked end to end, not taken from the kernel. The target critic's weights differ
from the local critic's (perturbed), so a mix-up of the two would show.

Cases: the reference's own N = 32 batch (tests/golden/learn_ac_iqn.npz, B = 64, its captured taus, the seeded
initial weights) and a B = 4096 random batch (the bench shape: 2048 rounds over 256 workgroups, the partials
reduced by asvrl_partial_sums).

Bars, fixed up front: loss and gradient norm within 1e-4 rel.; every critic gradient tensor element-wise within
min(2e-4, max(1e-4, 3 x the restatement's own f32 spread)) of its scale (max |g|) and within 1.5e-4 relative L2.
The element bar may exceed 1e-4 only where the restatement's own f32 evaluation (critic_step_bf16(dtype=float32),
printed beside each tensor) already spreads that far: bf16 rounding boundaries turn an f32-vs-f64 summation
difference into whole-ulp operand changes, so any f32 implementation of these rounding points shows that floor
(measured r05b at B = 4096: cos_embedding.bias f32 spread 1.64e-4). This pins the benched arithmetic itself (its
indexing, stage-ahead buffers, the in-launch target pass and the reductions): an indexing slip that moves the loss
by 1 % moves whole gradient tensors by far more.
"""
import numpy as np
import pytest
import torch

from oracle import env_oracle as eo
from oracle import learn_ref as lr

pytestmark = pytest.mark.gpu

BAR = 1e-4         # loss, gradient norm
BAR_ELEM_MAX = 2e-4   # per-tensor max |error| / max |g| ceiling (the floor is 1e-4, raised only to 3x the f32 spread)
BAR_L2 = 1.5e-4    # per-tensor relative L2
Q_L2 = 5e-5       # the in-launch target pass: |q_next - oracle| / |oracle| over the whole tensor (measured 1.7e-5,
                  # either kernel, B = 4096: v_cos_f32 vs the f64 cosine decides some bf16 cos operands)
Q_MAX = 5e-3      # and any single row (measured 1.89e-3 at B = 4096 with either kernel: rows whose bf16 cos / x / h1g
                  # operand or a ReLU pre-activation lands on the other side of a rounding boundary or kink)


def _split(x):
    B = x.shape[0]
    return (x[:, 0:7], x[:, 7:32].reshape(B, 5, 5), x[:, 32:37])


def _run(rows, taus, N, weights=None, tq=True, variant=8):
    """The benched critic launch on rows [B][88] with taus (2, B, N). Returns (grads, loss, q_next read by the
    update, q_next of the oracle, critic sd)."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_critic import critic_train_fused
    from distributional_rl_decision_and_control_amd.fused_mlp import actor_forward
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    B = rows.shape[0]
    ag = Agent(seed=100, agent_type="AC-IQN")
    loc, tgt = ag.policy_local, ag.policy_target
    with torch.no_grad():
        if weights is not None:
            for pol in (loc, tgt):
                for net in ("actor", "critic"):
                    for k, v in getattr(pol, net).state_dict().items():
                        v.copy_(torch.tensor(weights[net][k]))
        g = torch.Generator().manual_seed(7)
        for v in tgt.critic.parameters():   # a target distinct from the local critic
            v.add_((0.05 * float(v.abs().mean()) * torch.randn(v.shape, generator=g)).to(v.device))
    FusedAdam(loc.actor.parameters(), lr=1e-4, operands="bf16")
    co = FusedAdam(loc.critic.parameters(), lr=1e-4, operands="bf16")
    st = FusedACIQNState(loc, tgt, B, N, operands="bf16")
    critic, arena = loc.critic, st.arena
    co.grads.zero_()
    ns_rows = rows[:, 40:80]
    actor_forward(st.target_actor, ns_rows, st.na)   # the next actions (the launch's input a')
    torch.cuda.synchronize()
    tsd = {k: v.detach().cpu() for k, v in tgt.critic.state_dict().items()}
    x = rows.cpu().double()
    q_ref = lr.critic_forward_bf16(tsd, _split(x[:, 40:80]), st.na.cpu().double(), taus[0].cpu().double())
    if tq:
        st.q_next.fill_(float("nan"))   # written by the launch's target pass
        target = (st.target_trunk, taus[0], ns_rows, st.na)
    else:
        st.q_next.copy_(q_ref.reshape(-1).float().cuda())
        target = None
    from distributional_rl_decision_and_control_amd.fused_critic import fused_variant
    with fused_variant(variant):
        critic_train_fused(st.local_trunk, critic, taus[1], N, st.q_next.view(B, N), rows[:, 82], rows[:, 83], 0.99,
                           rows[:, 0:40], rows[:, 80:82], arena, tile_loss=st.tile_loss[0], encoders=True,
                           target=target)
    arena.scalar(st.tile_loss[0], st.losses[0:1])
    arena.flush()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu().double() for n, p in critic.named_parameters()}
    sd = {k: v.detach().cpu() for k, v in critic.state_dict().items()}
    return grads, float(st.losses[0].item()), st.q_next.view(B, N).cpu().double(), q_ref, sd


def _check(rows, taus, N, weights=None, tq=True, variant=8):
    g, loss, qn, q_ref, sd = _run(rows, taus, N, weights, tq, variant)
    qerr = float((qn - q_ref).abs().max() / (q_ref.abs().max() + 1e-30))
    ql2 = float((qn - q_ref).norm() / q_ref.norm())
    print(f"q_next (launch {'in-kernel target pass' if tq else 'oracle input'}) vs oracle: max err / scale {qerr:.2e}, "
          f"L2 {ql2:.2e}")
    assert ql2 < Q_L2 and qerr < Q_MAX, (ql2, qerr)
    x = rows.cpu().double()
    args = (sd, _split(x), x[:, 80:82], q_ref, x[:, 82], x[:, 83], taus[1].cpu().double())
    ref_loss, ref = lr.critic_step_bf16(*args)
    # the same rounding points in f32 arithmetic (CPU summation orders): the spread any f32 evaluation shows
    l32, g32 = lr.critic_step_bf16(*args, dtype=torch.float32)
    worst = 0.0
    bars = {}
    for n in ref:
        scale = float(ref[n].abs().max()) + 1e-30
        err = float((g[n] - ref[n]).abs().max()) / scale
        spread = float((g32[n].double() - ref[n]).abs().max()) / scale
        bars[n] = min(BAR_ELEM_MAX, max(1e-4, 3 * spread))
        worst = max(worst, err)
        l2 = float((g[n] - ref[n]).norm() / ref[n].norm())
        print(f"{n:28s} err/scale {err:.2e} (bar {bars[n]:.2e})  L2 {l2:.2e}  (f32 restatement {spread:.2e})  "
              f"scale {scale:.3e}")
    gn = float(torch.sqrt(sum((v * v).sum() for v in g.values())))
    rn = float(torch.sqrt(sum((v * v).sum() for v in ref.values())))
    print(f"loss kernel {loss:.7f} restatement {ref_loss:.7f} (f32 {l32:.7f}); norm {gn:.6f} vs {rn:.6f}; "
          f"worst {worst:.2e}")
    np.testing.assert_allclose(loss, ref_loss, rtol=BAR)
    np.testing.assert_allclose(gn, rn, rtol=BAR)
    bad = []
    for n in ref:
        scale = float(ref[n].abs().max()) + 1e-30
        err = float((g[n] - ref[n]).abs().max()) / scale
        # the whole tensor, not just its worst element: relative L2 error
        l2 = float((g[n] - ref[n]).norm() / ref[n].norm())
        if not (err < bars[n] and l2 < BAR_L2):
            bad.append((n, err, bars[n], l2))
    assert not bad, bad


VARIANTS = pytest.mark.parametrize("variant", [8, 4], ids=["two_waves_per_simd", "one_wave_per_simd"])


@VARIANTS
@pytest.mark.parametrize("tq", [True, False], ids=["tq_launch", "separate_target"])
def test_benched_critic_launch_on_the_reference_batch(tq, variant):
    from tests.test_learner_golden_gpu import _rows
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    rows = _rows(z, "n32/")
    taus = torch.from_numpy(z["n32/taus"][..., 0]).cuda().contiguous()
    weights = {net: {k[len(f"init/{net}/"):]: z[k] for k in z.keys() if k.startswith(f"init/{net}/")}
               for net in ("actor", "critic")}
    _check(rows, taus[:2], 32, weights, tq, variant)


@VARIANTS
@pytest.mark.parametrize("tq", [True, False], ids=["tq_launch", "separate_target"])
def test_benched_critic_launch_at_the_bench_shape(tq, variant):
    from tests.test_critic_fused_gpu import _batch
    B, N = 4096, 32
    rows, _ = _batch(B, 21)
    g = torch.Generator(device="cuda").manual_seed(22)
    taus = torch.rand(2, B, N, generator=g, device="cuda")
    _check(rows, taus, N, tq=tq, variant=variant)
