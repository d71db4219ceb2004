"""Export a trained policy as a float64 TorchScript module for the VRX deployment
(rfarl/scripts/save_model_to_torch_script.py, which traces the `*_dtype_double` twins of the
networks with f64 example inputs and saves `traced_{type}_model.pt`).

Here the same checkpoint files the trainer writes (`*_network_params.pth` +
`*_constructor_params.json`) are loaded with weights_only=True, converted to float64 and traced:

    python -m distributional_rl_decision_and_control_amd.scripts.save_model_to_torch_script \\
        --type AC_IQN --load-dir <run>/seed_0/... --out <dir>

AC_IQN / Rainbow trace forward(x) with x = (self (1,7), objects (1,5,5), mask (1,5)); IQN traces
forward(x, taus) with taus (1, K=32), as the reference's double IQN model does (IQN_model_dtype_double.py:75).
"""
import argparse
import os

import torch
import torch.nn as nn
from torch.nn.functional import relu

from ..policy.AC_IQN_model import Actor, encode_observation
from ..policy.IQN_model import IQN_Policy


def _example_state():
    return (torch.rand((1, 7), dtype=torch.float64), torch.rand((1, 5, 5), dtype=torch.float64),
            torch.rand((1, 5), dtype=torch.float64))


class _IQNDouble(nn.Module):
    """IQN_Policy.forward in float64 with the quantile fractions as an input (the reference's
    IQN_model_dtype_double.forward(x, taus))."""

    def __init__(self, net):
        super().__init__()
        self.net = net.double()
        self.register_buffer("pis", torch.arange(net.n, dtype=torch.float64).mul(torch.pi).view(1, 1, net.n))

    def forward(self, x, taus):
        n = self.net
        features = encode_observation(n.self_encoder, n.object_encoder, x, n.max_object_num, n.object_dimension,
                                      n.object_feature_dimension)
        B, K = taus.shape
        cos = torch.cos(taus.unsqueeze(-1) * self.pis).view(B * K, n.n)
        cos_features = relu(n.cos_embedding(cos)).view(B, K, n.concat_feature_dimension)
        f = (features.unsqueeze(1) * cos_features).view(B * K, n.concat_feature_dimension)
        f = relu(n.hidden_layer(f))
        f = relu(n.hidden_layer_2(f))
        return n.output_layer(f).view(B, K, n.action_size)


def export_torchscript(model_type, load_dir, out_dir, device="cpu"):
    """Trace the saved model of `model_type` in float64; returns the written path."""
    with torch.no_grad():   # inference graph only (also keeps the split-K training branch out)
        return _export(model_type, load_dir, out_dir, device)


def _export(model_type, load_dir, out_dir, device):
    out = os.path.join(out_dir, f"traced_{model_type}_model.pt")
    if model_type == "AC_IQN":
        model = Actor.load(load_dir, device).double().eval()
        traced = torch.jit.trace(model, (_example_state(),))
    elif model_type == "IQN":
        net = IQN_Policy.load(load_dir, device).eval()
        traced = torch.jit.trace(_IQNDouble(net).eval(), (_example_state(), torch.rand((1, 32), dtype=torch.float64)))
    elif model_type == "Rainbow":
        from ..policy.Rainbow_model import Rainbow_Policy
        model = Rainbow_Policy.load(load_dir, device).double().eval()
        traced = torch.jit.trace(model, (_example_state(),))
    else:
        raise NotImplementedError(f"TorchScript export of {model_type!r} (AC_IQN, IQN and Rainbow are supported)")
    traced.save(out)
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--type", required=True, choices=("AC_IQN", "IQN", "Rainbow"))
    ap.add_argument("--load-dir", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    print(export_torchscript(a.type, a.load_dir, a.out))


if __name__ == "__main__":
    main()
