"""DQN policy (rfarl/rfarl/policy/DQN_model.py:14-112): the non-distributional baseline BASELINE config 1
drives through train_RL_agents.py (plumbing only). Same layers, seeded init order,
state_dict keys and checkpoint files (network_params.pth + constructor_params.json)."""
import torch
import torch.nn as nn
from torch.nn.functional import relu

from .AC_IQN_model import _Saveable, encoder, encode_observation


class DQN_Policy(_Saveable, nn.Module):
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
        self.seed = torch.manual_seed(seed)  # DQN_model.py:38
        self.self_encoder = encoder(self_dimension, self_feature_dimension)
        self.object_encoder = encoder(object_dimension, object_feature_dimension)
        self.hidden_layer = nn.Linear(self.concat_feature_dimension, hidden_dimension)
        self.hidden_layer_2 = nn.Linear(hidden_dimension, hidden_dimension)
        self.output_layer = nn.Linear(hidden_dimension, action_size)

    def forward(self, x):  # DQN_model.py:50-74
        assert len(x) == 3, "The number of elements in state must be 3!"
        features = encode_observation(self.self_encoder, self.object_encoder, x, self.max_object_num,
                                      self.object_dimension, self.object_feature_dimension)
        features = relu(self.hidden_layer(features))
        features = relu(self.hidden_layer_2(features))
        return self.output_layer(features)

    def get_constructor_parameters(self):
        return dict(self_dimension=self.self_dimension, object_dimension=self.object_dimension,
                    max_object_num=self.max_object_num, self_feature_dimension=self.self_feature_dimension,
                    object_feature_dimension=self.object_feature_dimension,
                    concat_feature_dimension=self.concat_feature_dimension, hidden_dimension=self.hidden_dimension,
                    action_size=self.action_size, seed=self.seed_id)
