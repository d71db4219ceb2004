"""GPU: asvrl_linear_wgrad / asvrl_linear_wgrad_vec (csrc/asvrl_wgrad.hip), the Linear
weight-gradient reduction dW = dZ^T X, db = dZ.sum(0) (torch's nn.Linear backward,
AC_IQN_model.py:398-404), against f64 torch on the same bf16 inputs.

Small-integer inputs make every product and partial sum exact in f32, so the first test is
bit-exact and pins the transposed-LDS operand maps; random inputs are checked to 1e-5 of the
output scale (f32 accumulation over up to 131072 rows)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(256, 64), (128, 256), (128, 128), (64, 64)]


def _run(dz, x, accumulate=False, dw=None, db=None):
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.fused_critic import linear_wgrad
    M, K = dz.shape[1], x.shape[1]
    dw = torch.zeros(M, K, device="cuda") if dw is None else dw
    db = torch.zeros(M, device="cuda") if db is None else db
    work = torch.empty(int(_abi.lib().asvrl_linear_wgrad_workspace(M, K)), device="cuda")
    linear_wgrad(dz, x, dw, db, work, accumulate=accumulate)
    torch.cuda.synchronize()
    return dw, db


@pytest.mark.parametrize("M,K", SHAPES)
def test_wgrad_exact_on_integers(M, K):
    R = 2048
    g = torch.Generator(device="cuda").manual_seed(M + K)
    dz = torch.randint(-3, 4, (R, M), generator=g, device="cuda").to(torch.bfloat16)
    x = torch.randint(-3, 4, (R, K), generator=g, device="cuda").to(torch.bfloat16)
    dw, db = _run(dz, x)
    ref = dz.double().t() @ x.double()
    assert torch.equal(dw.double(), ref)
    assert torch.equal(db.double(), dz.double().sum(0))


@pytest.mark.parametrize("M,K", SHAPES)
@pytest.mark.parametrize("R", [32, 4096 + 96, 131072])
def test_wgrad_random(M, K, R):
    g = torch.Generator(device="cuda").manual_seed(R)
    dz = torch.randn(R, M, generator=g, device="cuda").to(torch.bfloat16)
    x = torch.randn(R, K, generator=g, device="cuda").to(torch.bfloat16)
    dw, db = _run(dz, x)
    ref = dz.double().t() @ x.double()
    assert (dw.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    rb = dz.double().sum(0)
    assert (db.double() - rb).abs().max().item() <= 1e-5 * rb.abs().max().item()


def test_wgrad_strided_and_accumulate():
    """Operands as column slices of wider row-major buffers; accumulate=1 adds."""
    R, M, K = 4096, 128, 128
    g = torch.Generator(device="cuda").manual_seed(5)
    big_z = torch.randn(R, M + 64, generator=g, device="cuda").to(torch.bfloat16)
    big_x = torch.randn(R, K + 128, generator=g, device="cuda").to(torch.bfloat16)
    dz, x = big_z[:, 64:], big_x[:, :K]
    dw0 = torch.randn(M, K, generator=g, device="cuda")
    db0 = torch.randn(M, generator=g, device="cuda")
    dw, db = _run(dz, x, accumulate=True, dw=dw0.clone(), db=db0.clone())
    ref = dz.double().t() @ x.double() + dw0.double()
    assert (dw.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    assert (db.double() - (dz.double().sum(0) + db0.double())).abs().max().item() <= 1e-4


@pytest.mark.parametrize("K", [64, 128, 256])
def test_wgrad_vec(K):
    from distributional_rl_decision_and_control_amd.fused_critic import linear_wgrad_vec
    R = 131072
    g = torch.Generator(device="cuda").manual_seed(K)
    dq = torch.randn(R, generator=g, device="cuda")
    x = torch.randn(R, K, generator=g, device="cuda").to(torch.bfloat16)
    dw = torch.zeros(K, device="cuda")
    db = torch.zeros(1, device="cuda")
    work = torch.empty(256 * (K + 1), device="cuda")
    linear_wgrad_vec(dq, x, dw, db, work)
    ref = dq.double() @ x.double()
    assert (dw.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    assert abs(db.item() - dq.double().sum().item()) <= 1e-4 * dq.abs().sum().item() * 1e-3


def test_partial_arena_is_bit_identical_to_per_layer_reduction():
    """PartialArena (partials of several layers, one asvrl_partial_sums launch) gives exactly
    the per-layer asvrl_linear_wgrad / _vec / asvrl_small_wgrad results (same partials, same
    fixed summation order), including more segments than one launch takes."""
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.fused_critic import PartialArena, linear_wgrad, linear_wgrad_vec
    from distributional_rl_decision_and_control_amd.fused_mlp import small_wgrad
    g = torch.Generator(device="cuda").manual_seed(9)
    R = 8192
    arena = PartialArena(32 << 20, "cuda")
    work = torch.empty(int(_abi.lib().asvrl_linear_wgrad_workspace(128, 256)), device="cuda")
    cases, outs_a, outs_b = [], [], []
    for (M, K) in SHAPES * 2 + [(256, 32)]:
        dz = torch.randn(R, M, generator=g, device="cuda").to(torch.bfloat16)
        x = torch.randn(R, K, generator=g, device="cuda").to(torch.bfloat16)
        wa, ba = torch.zeros(M, K, device="cuda"), torch.zeros(M, device="cuda")
        wb, bb = torch.zeros(M, K, device="cuda"), torch.zeros(M, device="cuda")
        linear_wgrad(dz, x, wa, ba, work)
        arena.linear(dz, x, wb, bb)
        outs_a += [wa, ba]
        outs_b += [wb, bb]
    dq = torch.randn(R, 2, generator=g, device="cuda")
    h = torch.randn(R, 128, generator=g, device="cuda").to(torch.bfloat16)
    wa, ba = torch.zeros(128, device="cuda"), torch.zeros(1, device="cuda")
    wb, bb = torch.zeros(128, device="cuda"), torch.zeros(1, device="cuda")
    linear_wgrad_vec(dq[:, 1], h, wa, ba, work)
    arena.vec(dq[:, 1], h, wb, bb)
    outs_a += [wa, ba]
    outs_b += [wb, bb]
    dzs = torch.randn(R, 128, generator=g, device="cuda")
    xs = torch.randn(R, 88, generator=g, device="cuda")[:, 80:82]
    wa, ba = torch.zeros(128, 2, device="cuda"), torch.zeros(128, device="cuda")
    wb, bb = torch.zeros(128, 2, device="cuda"), torch.zeros(128, device="cuda")
    small_wgrad(dzs, xs, wa, ba, torch.empty((R // 32) * 384, device="cuda"))
    arena.small(dzs, xs, wb, bb)
    outs_a += [wa, ba]
    outs_b += [wb, bb]
    arena.flush()
    torch.cuda.synchronize()
    for a, b in zip(outs_a, outs_b):
        assert torch.equal(a, b)
    ref = dzs.double().t() @ xs.double()
    assert (wa.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_partial_arena_scalar_segment():
    """A scalar segment (many groups, one output: the per-tile loss partials) is reduced by a
    whole workgroup in a fixed order: equal to an f64 sum within f32 rounding, deterministic."""
    from distributional_rl_decision_and_control_amd.fused_critic import PartialArena
    arena = PartialArena(1 << 20, "cuda")
    g = torch.Generator(device="cuda").manual_seed(4)
    parts = torch.randn(4096, generator=g, device="cuda")
    out1, out2 = torch.zeros(1, device="cuda"), torch.full((1,), 5.0, device="cuda")
    arena.scalar(parts, out1)
    arena.scalar(parts, out2, accumulate=True)
    arena.flush()
    again = torch.zeros(1, device="cuda")
    arena.scalar(parts, again)
    arena.flush()
    ref = parts.double().sum().item()
    assert abs(out1.item() - ref) <= 1e-5 * parts.abs().sum().item()
    assert abs(out2.item() - (ref + 5.0)) <= 1e-5 * parts.abs().sum().item() + 1e-6
    assert out1.item() == again.item()
