"""IQN policy (rfarl/rfarl/policy/IQN_model.py:14-146): same layers, init order, state_dict
keys and checkpoint files (network_params.pth + constructor_params.json)."""
import numpy as np
import torch
import torch.nn as nn
from torch.nn.functional import relu

from .AC_IQN_model import _Saveable, encoder, encode_observation


class IQN_Policy(_Saveable, nn.Module):
    _prefix = ""

    def __init__(self, self_dimension, object_dimension, max_object_num, self_feature_dimension,
                 object_feature_dimension, concat_feature_dimension, hidden_dimension, action_size, device="cpu",
                 seed=0):
        super().__init__()
        self.self_dimension = self_dimension
        self.object_dimension = object_dimension
        self.max_object_num = max_object_num
        self.self_feature_dimension = self_feature_dimension
        self.object_feature_dimension = object_feature_dimension
        self.concat_feature_dimension = concat_feature_dimension
        self.hidden_dimension = hidden_dimension
        self.action_size = action_size
        self.device = device
        self.seed_id = seed
        self.seed = torch.manual_seed(seed)  # IQN_model.py:39
        self.self_encoder = encoder(self_dimension, self_feature_dimension)
        self.object_encoder = encoder(object_dimension, object_feature_dimension)
        self.K = 32
        self.n = 64
        self.register_buffer("pis", torch.FloatTensor([np.pi * i for i in range(self.n)]).view(1, 1, self.n),
                             persistent=False)
        self.cos_embedding = nn.Linear(self.n, self.concat_feature_dimension)
        self.hidden_layer = nn.Linear(self.concat_feature_dimension, hidden_dimension)
        self.hidden_layer_2 = nn.Linear(hidden_dimension, hidden_dimension)
        self.output_layer = nn.Linear(hidden_dimension, action_size)

    def calc_cos(self, batch_size, num_tau=8, cvar=1.0, taus=None):  # IQN_model.py:56-72
        if taus is None:
            taus = torch.rand(batch_size, num_tau, device=self.pis.device).unsqueeze(-1)
        else:
            taus = taus.reshape(batch_size, num_tau, 1).to(self.pis.device, torch.float32)
        taus = taus * cvar
        return torch.cos(taus * self.pis), taus

    def forward(self, x, num_tau=8, cvar=1.0, taus=None):  # IQN_model.py:74-110
        assert len(x) == 3, "The number of elements in state must be 3!"
        features = encode_observation(self.self_encoder, self.object_encoder, x, self.max_object_num,
                                      self.object_dimension, self.object_feature_dimension)
        batch_size = features.shape[0]
        cos, taus = self.calc_cos(batch_size, num_tau, cvar, taus)
        cos = cos.view(batch_size * num_tau, self.n)
        cos_features = relu(self.cos_embedding(cos)).view(batch_size, num_tau, self.concat_feature_dimension)
        features = (features.unsqueeze(1) * cos_features).view(batch_size * num_tau, self.concat_feature_dimension)
        features = relu(self.hidden_layer(features))
        features = relu(self.hidden_layer_2(features))
        quantiles = self.output_layer(features)
        return quantiles.view(batch_size, num_tau, self.action_size), taus

    def get_constructor_parameters(self):
        return dict(self_dimension=self.self_dimension, object_dimension=self.object_dimension,
                    max_object_num=self.max_object_num, self_feature_dimension=self.self_feature_dimension,
                    object_feature_dimension=self.object_feature_dimension,
                    concat_feature_dimension=self.concat_feature_dimension, hidden_dimension=self.hidden_dimension,
                    action_size=self.action_size, seed=self.seed_id)
