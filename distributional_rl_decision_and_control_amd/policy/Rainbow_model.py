"""Rainbow (dueling NoisyNet C51) policy (rfarl/rfarl/policy/Rainbow_model.py:17-181): same
layers, init/noise draw order, state_dict keys and checkpoint files."""
import math

import torch
from torch import nn
from torch.nn import functional as F

from .AC_IQN_model import _Saveable, encoder, encode_observation


class NoisyLinear(nn.Module):
    """Factorised NoisyLinear with bias (Rainbow_model.py:17-53)."""

    def __init__(self, in_features, out_features, std_init=0.05):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.std_init = std_init
        self.weight_mu = nn.Parameter(torch.empty(out_features, in_features))
        self.weight_sigma = nn.Parameter(torch.empty(out_features, in_features))
        self.register_buffer("weight_epsilon", torch.empty(out_features, in_features))
        self.bias_mu = nn.Parameter(torch.empty(out_features))
        self.bias_sigma = nn.Parameter(torch.empty(out_features))
        self.register_buffer("bias_epsilon", torch.empty(out_features))
        self.reset_parameters()
        self.reset_noise()

    def reset_parameters(self):
        mu_range = 1 / math.sqrt(self.in_features)
        self.weight_mu.data.uniform_(-mu_range, mu_range)
        self.weight_sigma.data.fill_(self.std_init / math.sqrt(self.in_features))
        self.bias_mu.data.uniform_(-mu_range, mu_range)
        self.bias_sigma.data.fill_(self.std_init / math.sqrt(self.out_features))

    def _scale_noise(self, size):
        x = torch.randn(size, device=self.weight_mu.device)
        return x.sign().mul_(x.abs().sqrt_())

    def reset_noise(self):
        epsilon_in = self._scale_noise(self.in_features)
        epsilon_out = self._scale_noise(self.out_features)
        self.weight_epsilon.copy_(epsilon_out.ger(epsilon_in))
        self.bias_epsilon.copy_(epsilon_out)

    def forward(self, input):
        if self.training:
            return F.linear(input, self.weight_mu + self.weight_sigma * self.weight_epsilon,
                            self.bias_mu + self.bias_sigma * self.bias_epsilon)
        return F.linear(input, self.weight_mu, self.bias_mu)


class Rainbow_Policy(_Saveable, nn.Module):
    _prefix = ""

    def __init__(self, self_dimension, object_dimension, max_object_num, self_feature_dimension,
                 object_feature_dimension, concat_feature_dimension, hidden_dimension, action_size, atoms,
                 device="cpu", seed=0):
        super().__init__()
        self.self_dimension = self_dimension
        self.object_dimension = object_dimension
        self.max_object_num = max_object_num
        self.self_feature_dimension = self_feature_dimension
        self.object_feature_dimension = object_feature_dimension
        self.concat_feature_dimension = concat_feature_dimension
        self.hidden_dimension = hidden_dimension
        self.action_size = action_size
        self.atoms = atoms
        self.device = device
        self.seed_id = seed
        self.seed = torch.manual_seed(seed)  # Rainbow_model.py:82
        self.self_encoder = encoder(self_dimension, self_feature_dimension)
        self.object_encoder = encoder(object_dimension, object_feature_dimension)
        self.hidden_layer_v = NoisyLinear(self.concat_feature_dimension, hidden_dimension)
        self.hidden_layer_a = NoisyLinear(self.concat_feature_dimension, hidden_dimension)
        self.hidden_layer_v_2 = NoisyLinear(hidden_dimension, hidden_dimension)
        self.hidden_layer_a_2 = NoisyLinear(hidden_dimension, hidden_dimension)
        self.output_layer_v = NoisyLinear(hidden_dimension, self.atoms)
        self.output_layer_a = NoisyLinear(hidden_dimension, action_size * self.atoms)

    def forward(self, x, log=False):  # Rainbow_model.py:97-139
        assert len(x) == 3, "The number of elements in state must be 3!"
        features = encode_observation(self.self_encoder, self.object_encoder, x, self.max_object_num,
                                      self.object_dimension, self.object_feature_dimension)
        fv = F.relu(self.hidden_layer_v(features))
        fv = F.relu(self.hidden_layer_v_2(fv))
        v = self.output_layer_v(fv)
        fa = F.relu(self.hidden_layer_a(features))
        fa = F.relu(self.hidden_layer_a_2(fa))
        a = self.output_layer_a(fa)
        v, a = v.view(-1, 1, self.atoms), a.view(-1, self.action_size, self.atoms)
        q = v + a - a.mean(1, keepdim=True)
        return F.log_softmax(q, dim=2) if log else F.softmax(q, dim=2)

    def reset_noise(self):
        for name, module in self.named_children():
            if "hidden_layer" in name or "output_layer" in name:
                module.reset_noise()

    def get_constructor_parameters(self):
        return dict(self_dimension=self.self_dimension, object_dimension=self.object_dimension,
                    max_object_num=self.max_object_num, self_feature_dimension=self.self_feature_dimension,
                    object_feature_dimension=self.object_feature_dimension,
                    concat_feature_dimension=self.concat_feature_dimension, hidden_dimension=self.hidden_dimension,
                    action_size=self.action_size, atoms=self.atoms, seed=self.seed_id)
