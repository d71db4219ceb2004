"""GPU: asvrl_actor_grads (csrc/asvrl_wgrad.hip) -- every Actor gradient (AC_IQN_model.py:284-321 layers,
agent.py:424-426 actor_loss.backward()), the actor loss, the squared-norm partials and the Adam step count in
one launch, each 32 x 32 tile reduced over row splits by the split that arrives last.

Reference: an f64 restatement of the same sums from the same stored operands (dW = dZ^T X, db = dZ.sum(0),
the encoder image folded over the five object copies). Bar: |err| <= 1e-5 * sum_r |dz_r||x_r| per element
(f32 accumulation of at most B terms), the norm partials within 1e-6 of the f64 sum of squares, bit-identical
results on repeated launches (the arrival order changes nothing; counters are left zero)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(operands, B, seed):
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.fused_mlp import ActorBuffers, ActorGrads
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import AC_IQN_Policy
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    pol = AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1, 1], [-1, 1]], device="cuda", seed=100)
    actor = pol.actor
    opt = FusedAdam(actor.parameters(), operands=operands)   # contiguous .grad views
    ab = ActorBuffers(B, "cuda", operands)
    g = torch.Generator(device="cuda").manual_seed(seed)
    dt = _abi.operand_dtype(operands)

    def act(t, scale, relu):
        v = torch.randn(t.shape, generator=g, device="cuda") * scale
        t.copy_((v.clamp_min(0) if relu else v).to(dt))

    act(ab.xb, 3.0, False)
    act(ab.h0, 1.0, True)
    act(ab.h1, 1.0, True)
    act(ab.h2, 1.0, True)
    act(ab.dz2, 1e-3, False)
    act(ab.dz1, 1e-3, False)
    act(ab.dz0, 1e-3, False)
    ab.dout.copy_(torch.randn(B, 2, generator=g, device="cuda") * 1e-3)
    ws = ActorGrads(B, "cuda", operands)
    return actor, opt, ab, ws


def _reference(ab):
    d = lambda t: t.double()
    ref, bound = {}, {}

    def lin(name, dz, x):
        ref[name + ".weight"] = d(dz).T @ d(x)
        ref[name + ".bias"] = d(dz).sum(0)
        bound[name + ".weight"] = d(dz).abs().T @ d(x).abs()
        bound[name + ".bias"] = d(dz).abs().sum(0)

    lin("hidden_layer", ab.dz1, ab.h0)
    lin("hidden_layer_2", ab.dz2, ab.h1)
    lin("output_layer", ab.dout, ab.h2)
    E, Eb = d(ab.dz0).T @ d(ab.xb), d(ab.dz0).sum(0)
    A, Ab = d(ab.dz0).abs().T @ d(ab.xb).abs(), d(ab.dz0).abs().sum(0)

    def obj(M, rows_only):
        if rows_only:
            return sum(M[56 + 40 * o:96 + 40 * o] for o in range(5))
        return sum(M[56 + 40 * o:96 + 40 * o, 7 + 5 * o:12 + 5 * o] for o in range(5))

    ref["self_encoder.0.weight"], bound["self_encoder.0.weight"] = E[0:56, 0:7], A[0:56, 0:7]
    ref["self_encoder.0.bias"], bound["self_encoder.0.bias"] = Eb[0:56], Ab[0:56]
    ref["object_encoder.0.weight"], bound["object_encoder.0.weight"] = obj(E, False), obj(A, False)
    ref["object_encoder.0.bias"], bound["object_encoder.0.bias"] = obj(Eb, True), obj(Ab, True)
    return ref, bound


@pytest.mark.parametrize("operands", ["bf16", "f32"])
@pytest.mark.parametrize("B", [4096, 544, 32])
def test_actor_grads_match_f64_sums(operands, B):
    from distributional_rl_decision_and_control_amd.fused_mlp import actor_grads
    actor, opt, ab, ws = _setup(operands, B, seed=B)
    tile_loss = torch.randn(B * 32 // 32, device="cuda")
    loss = torch.zeros(1, device="cuda")
    step = torch.zeros(1, device="cuda")
    actor_grads(ws, ab, actor, tile_loss, loss, step=step)
    torch.cuda.synchronize()
    ref, bound = _reference(ab)
    params = dict(actor.named_parameters())
    sq = 0.0
    for name, r in ref.items():
        got = params[name].grad.double()
        assert got.shape == r.shape, name
        err = (got - r).abs()
        assert bool((err <= 1e-5 * bound[name] + 1e-30).all()), (name, err.max().item())
        sq += float((got ** 2).sum())
    assert abs(float(ws.norm_parts.sum()) - sq) <= 1e-6 * sq
    assert abs(loss.item() - tile_loss.double().sum().item()) <= 1e-5 * tile_loss.abs().sum().item()
    assert step.item() == 1.0
    assert int(ws.counters.abs().sum()) == 0


@pytest.mark.parametrize("operands", ["bf16", "f32"])
def test_actor_grads_repeatable(operands):
    """Launches in a row give bit-identical gradients and norm partials whatever the arrival order."""
    from distributional_rl_decision_and_control_amd.fused_mlp import actor_grads
    actor, opt, ab, ws = _setup(operands, 4096, seed=7)
    first = None
    for _ in range(4):
        opt.grads.flat.fill_(float("nan"))
        actor_grads(ws, ab, actor)
        now = (opt.grads.flat.clone(), ws.norm_parts.clone())
        if first is None:
            first = now
        else:
            assert torch.equal(now[0], first[0]) and torch.equal(now[1], first[1])
    assert not torch.isnan(first[0]).any()
    assert int(ws.counters.abs().sum()) == 0


def test_actor_grads_argument_checks():
    import ctypes as C
    from distributional_rl_decision_and_control_amd import _abi
    L = _abi.lib()
    io = _abi.AsvActorGradIO()
    assert L.asvrl_actor_grads(C.byref(io), None) != 0
    assert b"null" in L.asvrl_last_error()

