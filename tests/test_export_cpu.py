"""CPU: float64 TorchScript export of trained policies (rfarl/scripts/save_model_to_torch_script.py).
A seeded network is saved in the trainer's checkpoint format, exported, re-loaded (our own file)
and compared with the f32 module on the same f64 inputs: 1e-5 relative (f32 vs f64 arithmetic)."""
import numpy as np
import torch


def _state(n, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, 7, generator=g, dtype=torch.float64), torch.randn(n, 5, 5, generator=g, dtype=torch.float64),
            (torch.rand(n, 5, generator=g) > 0.3).double())


def test_export_ac_iqn_actor(tmp_path):
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import AC_IQN_Policy
    from distributional_rl_decision_and_control_amd.scripts.save_model_to_torch_script import export_torchscript
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    pol = AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1, 1], [-1, 1]], device="cpu", seed=7)
    pol.save(str(tmp_path))
    path = export_torchscript("AC_IQN", str(tmp_path), str(tmp_path))
    ts = torch.jit.load(path)
    x = _state(16, 1)
    out = ts(x)
    assert out.dtype == torch.float64 and out.shape == (16, 2)
    with torch.no_grad():
        ref = pol.actor(tuple(t.float() for t in x)).double()
    np.testing.assert_allclose(out.detach().numpy(), ref.numpy(), rtol=1e-5, atol=1e-6)


def test_export_iqn(tmp_path):
    from distributional_rl_decision_and_control_amd.policy.IQN_model import IQN_Policy
    from distributional_rl_decision_and_control_amd.scripts.save_model_to_torch_script import export_torchscript
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    net = IQN_Policy(**DEFAULT_NET, action_size=25, device="cpu", seed=3)
    net.save(str(tmp_path))
    ts = torch.jit.load(export_torchscript("IQN", str(tmp_path), str(tmp_path)))
    x = _state(4, 2)
    taus = torch.rand(4, 32, dtype=torch.float64)
    out = ts(x, taus)
    assert out.dtype == torch.float64 and out.shape == (4, 32, 25)
    with torch.no_grad():
        ref, _ = net(tuple(t.float() for t in x), 32, taus=taus.float().unsqueeze(-1))
    np.testing.assert_allclose(out.detach().numpy(), ref.double().numpy(), rtol=1e-4, atol=1e-5)
