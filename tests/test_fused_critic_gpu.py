"""GPU: the fused MFMA critic (csrc/asvrl_critic.hip) against a plain torch fp32 restatement of
Critic.forward / the quantile-Huber critic loss / the actor loss (AC_IQN_model.py:410-480,
agent.py:395-427). The kernel computes in bf16 with f32 accumulation, so the tolerances are
bf16-sized: outputs within 2% of the output scale, gradients with cosine similarity > 0.995
and norms within 3%."""
import numpy as np
import pytest
import torch

from oracle import learn_ref as lr

pytestmark = pytest.mark.gpu


def _setup(B, N, seed=0):
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import Critic
    torch.manual_seed(seed)
    critic = Critic(7, 5, 5, 56, 40, 256, 128, 2, "cuda", 101).cuda()
    g = torch.Generator(device="cuda").manual_seed(seed)
    s = (torch.randn(B, 7, generator=g, device="cuda") * 3, torch.randn(B, 5, 5, generator=g, device="cuda") * 3,
         (torch.rand(B, 5, generator=g, device="cuda") > 0.3).float())
    a = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
    taus = torch.rand(B, N, generator=g, device="cuda")
    return critic, s, a, taus


def _features(critic, s, a):
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import encode_observation
    F = encode_observation(critic.self_encoder, critic.object_encoder, s, 5, 5, 40)
    G = critic.action_encoder(a)
    return F, G


def _cos(x, y):
    x, y = x.reshape(-1).double(), y.reshape(-1).double()
    return float((x @ y) / (x.norm() * y.norm() + 1e-30))


def test_pack_kernel_matches_fragment_index():
    """asvrl_critic_pack writes exactly the frag_index gathers (bit-exact bf16 images)."""
    from distributional_rl_decision_and_control_amd.fused_critic import CriticPack
    critic, _, _, _ = _setup(64, 8)
    pack = CriticPack(critic)
    torch.cuda.synchronize()
    ref = pack.reference_images()
    for name in ("wc", "w1", "w2", "w2t", "w1t"):
        assert torch.equal(getattr(pack, name), ref[name]), name
    with torch.no_grad():
        critic.hidden_layer.weight.mul_(-0.5)
    pack.refresh()
    ref = pack.reference_images()
    assert torch.equal(pack.w1, ref["w1"]) and torch.equal(pack.w1t, ref["w1t"])


@pytest.mark.parametrize("B,N", [(64, 8), (256, 32), (4096, 32)])
def test_fused_forward(B, N):
    from distributional_rl_decision_and_control_amd.fused_critic import CriticPack, critic_forward
    critic, s, a, taus = _setup(B, N)
    with torch.no_grad():
        q_ref, _ = critic(s, a, N, taus=taus.unsqueeze(-1))
        F, G = _features(critic, s, a)
        q = critic_forward(CriticPack(critic), F.contiguous(), G.contiguous(), taus.contiguous(), N)
    err = (q - q_ref).abs().max().item() / q_ref.abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("B", [1, 37, 4096])
def test_forward_launch_matches_in_launch_target_pass(B):
    """asvrl_critic_forward (critic_kernel<FWD>) against the fused launch's in-launch target pass
    (asvrl_critic_train_fused_tq with kernel variant 4: the same FWD tile compiled into the other file, its q_next written for the
    fused shape's rows): every row bit-identical, B = 1 and 37 (a partial launch) and 4096. (Round 4 also
    measured a two-tiles-per-wave FWD kernel, one wave per SIMD, against this one: 36 vs 26 us, dropped,
    profiles/r04u_fwd_two_tiles_ab.txt.)"""
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState, target_q
    from distributional_rl_decision_and_control_amd.fused_critic import critic_forward
    from tests.test_critic_fused_gpu import _batch
    Bp = max(64, -(-B // 64) * 64)   # the fused launch's shape; the forward alone runs on the first B rows
    rows, _ = _batch(Bp, 9)
    taus = torch.rand(Bp, 32, generator=torch.Generator(device="cuda").manual_seed(B), device="cuda")
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    ag = Agent(seed=3, agent_type="AC-IQN")
    FusedAdam(ag.policy_local.actor.parameters(), lr=1e-4)
    FusedAdam(ag.policy_local.critic.parameters(), lr=1e-4)   # contiguous .grad (the fused launch's encoders)
    st = FusedACIQNState(ag.policy_local, ag.policy_target, Bp, 32)
    target_q(st, rows, taus, st.q_next, st.na)   # the target actor's a' (and q_next by the two-tile kernel)
    q2 = critic_forward(st.target_trunk, None, None, taus[:B].contiguous(), 32, obs=rows[:B, 40:80],
                        act=st.na[:B])
    # the one-tile code path: the fused launch's target pass
    from distributional_rl_decision_and_control_amd.fused_critic import critic_train_fused
    from distributional_rl_decision_and_control_amd.fused_critic import fused_variant
    q1 = torch.full_like(st.q_next, float("nan"))
    with fused_variant(4):   # the kernel whose target pass IS this tile (variant 8: tests/test_critic_fused8_gpu.py)
        critic_train_fused(st.local_trunk, ag.policy_local.critic, taus, 32, q1.view(Bp, 32), rows[:, 82], rows[:, 83],
                           0.99, rows[:, 0:40], rows[:, 80:82], st.arena, tile_loss=st.tile_loss[0], encoders=True,
                           target=(st.target_trunk, taus, rows[:, 40:80], st.na))
    torch.cuda.synchronize()
    assert torch.isfinite(q2).all()
    assert torch.equal(q2.reshape(-1), q1.view(Bp, 32)[:B].reshape(-1))


@pytest.mark.parametrize("B,N", [(64, 8), (256, 16), (1024, 32)])
def test_encoders_in_kernel_match_torch(B, N):
    """Observation rows + actions instead of F / G: the trunk kernels run the critic's encoders
    (observation_processor, action_encoder) in f32 in their prologue; q matches torch fp32 and
    the F / G path."""
    from distributional_rl_decision_and_control_amd.fused_critic import CriticPack, critic_forward
    critic, s, a, taus = _setup(B, N, seed=3)
    rows = torch.zeros(B, 88, device="cuda")
    rows[:, 0:7], rows[:, 7:32], rows[:, 32:37] = s[0], s[1].reshape(B, 25), s[2]
    rows[:, 80:82] = a
    pack = CriticPack(critic)
    with torch.no_grad():
        q_ref, _ = critic(s, a, N, taus=taus.unsqueeze(-1))
        F, G = _features(critic, s, a)
        q_fg = critic_forward(pack, F.contiguous(), G.contiguous(), taus.contiguous(), N)
        q_obs = critic_forward(pack, None, None, taus.contiguous(), N, obs=rows[:, 0:40], act=rows[:, 80:82])
    scale = q_ref.abs().max().item()
    assert (q_obs - q_ref).abs().max().item() / scale < 2e-2
    assert (q_obs - q_fg).abs().max().item() / scale < 1e-2


@pytest.mark.parametrize("B,N,Np", [(64, 8, 8), (512, 32, 32)])
def test_fused_train_gradients(B, N, Np):
    from distributional_rl_decision_and_control_amd.fused_critic import (CriticPack, TrainBuffers, critic_train,
                                                                          trunk_weight_grads)
    from distributional_rl_decision_and_control_amd.learner import FlatGrads
    critic, s, a, taus = _setup(B, N, seed=1)
    g = torch.Generator(device="cuda").manual_seed(7)
    qt = (torch.randn(B, Np, generator=g, device="cuda") * 0.5).contiguous()
    # reference: fp32 autograd through the torch modules
    params = list(critic.parameters())
    q_ref, _ = critic(s, a, N, taus=taus.unsqueeze(-1))
    loss_ref = lr.quantile_huber(qt, q_ref, taus.unsqueeze(-1))
    grads_ref = torch.autograd.grad(loss_ref, params)
    # fused
    fg = FlatGrads(critic.parameters())
    fg.zero_()
    bufs = TrainBuffers(B, N, "cuda")
    F, G = _features(critic, s, a)
    loss = critic_train(CriticPack(critic), F.detach().contiguous(), G.detach().contiguous(), taus.contiguous(),
                        qt, bufs)
    trunk_weight_grads(critic, bufs)
    torch.autograd.backward([F, G], [bufs.dF, bufs.dG])
    assert abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()) < 1e-2
    names = [n for n, _ in critic.named_parameters()]
    for n, p, gr in zip(names, params, grads_ref):
        c = _cos(p.grad, gr)
        ratio = p.grad.norm().item() / max(gr.norm().item(), 1e-30)
        assert c > 0.995 and abs(ratio - 1) < 0.03, (n, c, ratio)


@pytest.mark.parametrize("B,N", [(64, 8), (512, 32)])
def test_fused_actor_gradient(B, N):
    from distributional_rl_decision_and_control_amd.fused_critic import CriticPack, critic_actor_grad
    critic, s, a, taus = _setup(B, N, seed=2)
    a = a.clone().requires_grad_(True)
    q_ref, _ = critic(s, a, N, taus=taus.unsqueeze(-1))
    (-q_ref.mean()).backward()
    da_ref = a.grad.clone()
    a2 = a.detach().clone().requires_grad_(True)
    F, G = _features(critic, s, a2)
    q = torch.empty(B * N, device="cuda")
    dG = torch.empty(B, 128, device="cuda")
    critic_actor_grad(CriticPack(critic), F.detach().contiguous(), G.detach().contiguous(), taus.contiguous(), N, q, dG)
    (da,) = torch.autograd.grad(G, a2, grad_outputs=dG)
    assert abs(q.mean().item() - q_ref.mean().item()) / q_ref.abs().mean().item() < 2e-2
    c = _cos(da, da_ref)
    assert c > 0.995, c
    assert abs(da.norm().item() / da_ref.norm().item() - 1) < 0.03


def test_fused_update_tracks_fp32_update():
    """Ten VecTrainer-shaped AC-IQN updates (B=512, N=32): the product learner (ac_iqn_update_fused2, bf16
    operands) follows the fp32 torch restatement (learner.ac_iqn_update, torch.optim.Adam) on identical
    replay rows and taus. Bar: losses within 3 % (+2e-3 absolute) at every step."""
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState, ac_iqn_update_fused2
    from distributional_rl_decision_and_control_amd.learner import FlatGrads, FusedAdam, ac_iqn_update
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import AC_IQN_Policy
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    B, N = 512, 32

    def nets():
        return [AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1, 1], [-1, 1]], device="cuda", seed=100)
                for _ in range(2)]

    loc, tgt = nets()
    cg, ag = FlatGrads(loc.critic.parameters()), FlatGrads(loc.actor.parameters())
    ao, co = torch.optim.Adam(loc.actor.parameters(), lr=1e-4), torch.optim.Adam(loc.critic.parameters(), lr=1e-4)
    floc, ftgt = nets()
    fao, fco = FusedAdam(floc.actor.parameters(), lr=1e-4), FusedAdam(floc.critic.parameters(), lr=1e-4)
    st = FusedACIQNState(floc, ftgt, B, N)
    g = torch.Generator(device="cuda").manual_seed(3)
    la, lb = [], []
    for _ in range(10):
        rows = torch.zeros(B, 88, device="cuda")
        for c in (0, 40):
            rows[:, c:c + 32] = torch.randn(B, 32, generator=g, device="cuda") * 3
            rows[:, c + 32:c + 37] = (torch.rand(B, 5, generator=g, device="cuda") > 0.3).float()
        rows[:, 80:82] = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
        rows[:, 82] = torch.randn(B, generator=g, device="cuda")
        rows[:, 83] = (torch.rand(B, generator=g, device="cuda") > 0.9).float()
        taus = torch.rand(3, B, N, generator=g, device="cuda")

        def obs(c):
            return rows[:, c:c + 7], rows[:, c + 7:c + 32].reshape(B, 5, 5), rows[:, c + 32:c + 37]
        out_a = ac_iqn_update(loc, tgt, ao, co, cg, ag, obs(0), rows[:, 80:82], rows[:, 82:83], obs(40),
                              rows[:, 83:84], num_tau=N, taus=tuple(t.unsqueeze(-1) for t in taus))
        out_b = ac_iqn_update_fused2(st, floc, fao, fco, fco.grads, fao.grads, rows, taus=taus)
        la.append([out_a[0].item(), out_a[1].item()])
        lb.append([out_b[0].item(), out_b[1].item()])
    la, lb = np.array(la), np.array(lb)
    np.testing.assert_allclose(lb, la, rtol=3e-2, atol=2e-3)


@pytest.mark.parametrize("B,N", [(256, 32), (512, 8)])
def test_train_output_layer_grad_in_kernel(B, N):
    """wout_part: the TRAIN kernel reduces output_layer's dW = sum dq h2 and db = sum dq over each
    32-row tile from f32 registers, then over the workgroup's tiles in LDS (h2 and dq stay on chip);
    the summed partials match the fp32
    autograd gradient (and the bf16-h2 reduction path) of the same launch inputs."""
    from distributional_rl_decision_and_control_amd.fused_critic import (CriticPack, TrainBuffers, critic_train,
                                                                          wout_groups)
    critic, s, a, taus = _setup(B, N, seed=4)
    g = torch.Generator(device="cuda").manual_seed(9)
    qt = (torch.randn(B, N, generator=g, device="cuda") * 0.5).contiguous()
    q_ref, _ = critic(s, a, N, taus=taus.unsqueeze(-1))
    loss_ref = lr.quantile_huber(qt, q_ref, taus.unsqueeze(-1))
    gw_ref, gb_ref = torch.autograd.grad(loss_ref, [critic.output_layer.weight, critic.output_layer.bias])
    F, G = _features(critic, s, a)
    pack = CriticPack(critic)
    bufs = TrainBuffers(B, N, "cuda")
    tiles = wout_groups(B, N)
    part = torch.full((tiles * 129,), float("nan"), device="cuda")
    critic_train(pack, F.detach().contiguous(), G.detach().contiguous(), taus.contiguous(), qt, bufs,
                 wout_part=part)
    p = part.view(tiles, 129).sum(0)
    gw, gb = p[:128], p[128]
    assert torch.isfinite(p).all()
    assert _cos(gw, gw_ref.reshape(-1)) > 0.999 and abs(gw.norm().item() / gw_ref.norm().item() - 1) < 0.02
    assert abs(gb.item() - gb_ref.item()) <= 1e-3 * abs(gb_ref.item()) + 1e-6
    # the same launch without wout_part: bf16 h2 + dq rows reduced on the host side
    critic_train(pack, F.detach().contiguous(), G.detach().contiguous(), taus.contiguous(), qt, bufs)
    gw2 = (bufs.dq[:, None] * bufs.h2.float()).sum(0)
    assert _cos(gw, gw2) > 0.999
    torch.testing.assert_close(gb, bufs.dq.sum(), rtol=1e-4, atol=1e-7)
