"""GPU: the hand-written Rainbow learner (fused_rainbow.FusedRainbow, f32-operand build libasvrl_f32.so)
pinned to the reference's own train_Rainbow (agent.py:597-641, Rainbow_model.py:17-139) at the default
network size, through the drop-in Agent.train_Rainbow.

Fixture: tests/golden/learn_rainbow_full.npz (tools/capture_oracle.py capture_rainbow_full, run against
/root/reference in the build container): both networks from oracle.learn_ref.synthetic_rainbow_state(seed)
(numpy, bit-exact), a B = 64 batch with the projection's edge cases (exact-integer b, clamping, terminal),
IS weights, and the target noise reset_noise() drew inside the reference's step, injected here
(reset_target_noise=False). Bars: per-sample loss (= the priorities) 1e-5 rel.; the double-Q argmax
exact on >= 63 of 64 rows (ties within 1e-5 may flip) and p(s', a*) 1e-5; the pre-clip gradient norm
1e-5 rel.; the clipped gradient the optimizer applies, per parameter (full tensors <= 4096 elements,
2048 sampled positions + whole-tensor sum / sum of squares otherwise), within 1e-5 of the tensor's max
|g| (+1e-4 rel.); the parameters after the Adam step within 1e-4 rel. / 2e-6 abs."""
import numpy as np
import pytest
import torch

from oracle import env_oracle as eo
from oracle import learn_ref as lr

pytestmark = pytest.mark.gpu


def _agent_on_fixture(z):
    from distributional_rl_decision_and_control_amd.agent import Agent
    ag = Agent(seed=100, agent_type="Rainbow")
    assert ag.learner == "fused-f32"
    sd = lr.synthetic_rainbow_state(int(z["seed"][0]))
    with torch.no_grad():
        for net in (ag.policy_local, ag.policy_target):
            for k, v in net.state_dict().items():
                v.copy_(torch.from_numpy(sd[k]))
        tsd = ag.policy_target.state_dict()
        for name, _, _ in lr.RAINBOW_NOISY:   # the reference's reset_noise draw inside train
            we, be = lr.noisy_epsilon(z["target_eps_in/" + name], z["target_eps_out/" + name])
            tsd[name + ".weight_epsilon"].copy_(torch.from_numpy(we))
            tsd[name + ".bias_epsilon"].copy_(torch.from_numpy(be))
    dev = ag.device
    t = lambda k: torch.tensor(z[k], device=dev)  # noqa: E731
    batch = (np.arange(64), (t("s_self"), t("s_obj"), t("s_mask")), t("actions").long(), t("returns"),
             (t("ns_self"), t("ns_obj"), t("ns_mask")), t("nonterminal"), t("weights"))
    ag.memory.sample = lambda bs: batch
    return ag


def test_fused_rainbow_learner_matches_reference_train_rainbow():
    z = np.load(eo.GOLDEN + "/learn_rainbow_full.npz")
    ag = _agent_on_fixture(z)
    pr = []
    ag.memory.update_priorities = lambda i, p: pr.append(np.array(p))
    loss = ag.train_Rainbow(reset_target_noise=False)
    st = ag._fused[1]
    assert st is not None and st.img.L is not None, "the kernel learner must run (default dims)"
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss, z["loss"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(pr[0], z["priorities"], rtol=1e-5, atol=1e-6)
    a_star = st.a_star.cpu().numpy()
    assert (a_star == z["argmax_ns"]).sum() >= 63
    ok = a_star == z["argmax_ns"]
    np.testing.assert_allclose(st.p_star.cpu().numpy()[ok], z["pns_a"][ok], rtol=1e-5, atol=1e-7)
    # pre-clip norm: the learner's reduction forms it in f64 from the f32 gradient
    gsq = float(sum(float((p.grad.double() ** 2).sum()) for p in ag.policy_local.parameters()))
    clip = min(1.0, 0.5 / (float(z["grad_norm"][0]) + 1e-6))
    np.testing.assert_allclose(np.sqrt(gsq) / clip, z["grad_norm"][0], rtol=1e-5)
    for n, p in ag.policy_local.named_parameters():
        g = p.grad.detach().reshape(-1).double().cpu().numpy()
        a = p.detach().reshape(-1).double().cpu().numpy()
        if "idx/" + n in z.files:
            ix = z["idx/" + n]
            gs, ss = z["gsum/" + n]
            scale = np.sqrt(ss / g.size)
            assert abs(g.sum() - gs) <= 1e-5 * np.sqrt(ss * g.size) + 1e-12, n
            np.testing.assert_allclose((g ** 2).sum(), ss, rtol=2e-5, err_msg=n)
            g, a = g[ix], a[ix]
        ref_g, ref_a = z["grad/" + n].astype(np.float64), z["after/" + n].astype(np.float64)
        tol = 1e-5 * np.abs(ref_g).max() + 1e-12
        np.testing.assert_allclose(g, ref_g, rtol=1e-4, atol=tol, err_msg=n)
        np.testing.assert_allclose(a, ref_a, rtol=1e-4, atol=2e-6, err_msg=n)


def test_train_rainbow_kernel_path_is_default_and_torch_path_agrees():
    """set_learner("torch") runs learner.rainbow_update (torch autograd + C51 kernel) on the same fixture:
    both learners meet the same reference (losses 1e-5), so the switch changes no semantics."""
    z = np.load(eo.GOLDEN + "/learn_rainbow_full.npz")
    ag = _agent_on_fixture(z)
    ag.set_learner("torch")
    ag.memory.update_priorities = lambda i, p: None
    loss = ag.train_Rainbow(reset_target_noise=False)
    assert ag._fused is None or ag._fused[1] is None
    np.testing.assert_allclose(loss, z["loss"], rtol=1e-5, atol=1e-6)
