"""AC-IQN actor / critic (rfarl/rfarl/policy/AC_IQN_model.py:16-516).

Same constructor arguments, layer names (state_dict keys), seeded initialisation order and
checkpoint files (actor_network_params.pth + actor_constructor_params.json, critic_...) as
the reference, so checkpoints move between the two. Differences are additive: forward()
accepts pre-drawn `taus` (parity tests, graph capture), and the object encoder treats a
missing object batch as all-masked (numerically identical, AC_IQN_model.py:293-294).
"""
import copy
import json
import os

import numpy as np
import torch
import torch.nn as nn
from torch.nn.functional import relu


def encoder(input_dimension, output_dimension):
    return nn.Sequential(nn.Linear(input_dimension, output_dimension), nn.ReLU())


def encode_observation(self_encoder, object_encoder, x, max_object_num, object_dimension, object_feature_dimension):
    """observation_processor's shared part (AC_IQN_model.py:284-308, IQN_model.py:76-96)."""
    x_1, x_2, x_2_mask = x
    batch_size = x_1.shape[0]
    f1 = self_encoder(x_1)
    if x_2 is None:
        f2 = torch.zeros((batch_size, max_object_num * object_feature_dimension), device=x_1.device, dtype=f1.dtype)
    else:
        f2 = object_encoder(x_2.reshape(batch_size * max_object_num, object_dimension))
        f2 = f2.view(batch_size, max_object_num, object_feature_dimension)
        f2 = f2.masked_fill(x_2_mask.unsqueeze(-1) < 0.5, 0.0)
        f2 = f2.reshape(batch_size, max_object_num * object_feature_dimension)
    return torch.cat((f1, f2), 1)


class AC_IQN_Policy:
    def __init__(self, self_dimension, object_dimension, max_object_num, self_feature_dimension,
                 object_feature_dimension, concat_feature_dimension, hidden_dimension, value_ranges_of_action,
                 device="cpu", seed=0):
        self.actor = Actor(self_dimension, object_dimension, max_object_num, self_feature_dimension,
                           object_feature_dimension, concat_feature_dimension, hidden_dimension,
                           value_ranges_of_action, device, seed).to(device)
        self.critic = Critic(self_dimension, object_dimension, max_object_num, self_feature_dimension,
                             object_feature_dimension, concat_feature_dimension, hidden_dimension,
                             len(value_ranges_of_action), device, seed + 1).to(device)

    def save(self, directory):
        self.actor.save(directory)
        self.critic.save(directory)

    @classmethod
    def load(cls, directory, device="cpu"):
        actor = Actor.load(directory, device)
        critic = Critic.load(directory, device)
        policy = cls(actor.self_dimension, actor.object_dimension, actor.max_object_num,
                     actor.self_feature_dimension, actor.object_feature_dimension, actor.concat_feature_dimension,
                     actor.hidden_dimension, actor.value_ranges_of_action, device=device)
        policy.actor = actor
        policy.critic = critic
        return policy


class _Saveable:
    _prefix = ""

    def save(self, directory):
        torch.save(self.state_dict(), os.path.join(directory, f"{self._prefix}network_params.pth"))
        with open(os.path.join(directory, f"{self._prefix}constructor_params.json"), mode="w") as f:
            json.dump(self.get_constructor_parameters(), f)

    @classmethod
    def load(cls, directory, device="cpu"):
        params = torch.load(os.path.join(directory, f"{cls._prefix}network_params.pth"), map_location=device,
                            weights_only=True)
        with open(os.path.join(directory, f"{cls._prefix}constructor_params.json"), mode="r") as f:
            ctor = json.load(f)
            ctor["device"] = device
        model = cls(**ctor)
        model.load_state_dict(params)
        model.to(device)
        return model


class Actor(_Saveable, nn.Module):
    _prefix = "actor_"

    def __init__(self, self_dimension, object_dimension, max_object_num, self_feature_dimension,
                 object_feature_dimension, concat_feature_dimension, hidden_dimension, value_ranges_of_action,
                 device="cpu", seed=0):
        super().__init__()
        self.self_dimension = self_dimension
        self.object_dimension = object_dimension
        self.max_object_num = max_object_num
        self.self_feature_dimension = self_feature_dimension
        self.object_feature_dimension = object_feature_dimension
        self.concat_feature_dimension = concat_feature_dimension
        self.hidden_dimension = hidden_dimension
        self.value_ranges_of_action = copy.deepcopy(value_ranges_of_action)
        self.action_dimension = len(self.value_ranges_of_action)
        self.device = device
        self.seed_id = seed
        self.seed = torch.manual_seed(seed)  # AC_IQN_model.py:269
        self.register_buffer("atan_scale", torch.tensor(2.0 / torch.pi), persistent=False)  # :271
        self.self_encoder = encoder(self_dimension, self_feature_dimension)
        self.object_encoder = encoder(object_dimension, object_feature_dimension)
        self.hidden_layer = nn.Linear(self.concat_feature_dimension, hidden_dimension)
        self.hidden_layer_2 = nn.Linear(hidden_dimension, hidden_dimension)
        self.output_layer = nn.Linear(hidden_dimension, self.action_dimension)

    def observation_processor(self, x):
        assert len(x) == 3, "The number of elements in state must be 3!"
        return encode_observation(self.self_encoder, self.object_encoder, x, self.max_object_num,
                                  self.object_dimension, self.object_feature_dimension)

    def forward(self, x):
        features = self.observation_processor(x)
        features = relu(self.hidden_layer(features))
        features = relu(self.hidden_layer_2(features))
        actions = self.output_layer(features)
        return self.atan_scale * torch.atan(actions)  # map to (-1, 1) (AC_IQN_model.py:321)

    def get_constructor_parameters(self):
        return dict(self_dimension=self.self_dimension, object_dimension=self.object_dimension,
                    max_object_num=self.max_object_num, self_feature_dimension=self.self_feature_dimension,
                    object_feature_dimension=self.object_feature_dimension,
                    concat_feature_dimension=self.concat_feature_dimension, hidden_dimension=self.hidden_dimension,
                    value_ranges_of_action=self.value_ranges_of_action, seed=self.seed_id)


class Critic(_Saveable, nn.Module):
    _prefix = "critic_"

    def __init__(self, self_dimension, object_dimension, max_object_num, self_feature_dimension,
                 object_feature_dimension, concat_feature_dimension, hidden_dimension, action_dimension,
                 device="cpu", seed=0):
        super().__init__()
        self.self_dimension = self_dimension
        self.object_dimension = object_dimension
        self.max_object_num = max_object_num
        self.self_feature_dimension = self_feature_dimension
        self.object_feature_dimension = object_feature_dimension
        self.concat_feature_dimension = concat_feature_dimension
        self.hidden_dimension = hidden_dimension
        self.action_dimension = action_dimension
        self.device = device
        self.seed_id = seed
        self.seed = torch.manual_seed(seed)  # AC_IQN_model.py:387
        self.K = 32
        self.n = 64
        self.self_encoder = encoder(self_dimension, self_feature_dimension)
        self.object_encoder = encoder(object_dimension, object_feature_dimension)
        self.register_buffer("pis", torch.FloatTensor([np.pi * i for i in range(self.n)]).view(1, 1, self.n),
                             persistent=False)
        self.cos_embedding = nn.Linear(self.n, self.concat_feature_dimension)
        self.action_encoder = encoder(self.action_dimension, hidden_dimension)
        self.hidden_layer = nn.Linear(self.concat_feature_dimension, hidden_dimension)
        self.hidden_layer_2 = nn.Linear(hidden_dimension, hidden_dimension)
        self.output_layer = nn.Linear(hidden_dimension, 1)

    def calc_cos(self, batch_size, num_tau=8, cvar=1.0, taus=None):
        """AC_IQN_model.py:410-426; `taus` (B, N, 1) may be supplied instead of torch.rand."""
        if taus is None:
            taus = torch.rand(batch_size, num_tau, device=self.pis.device).unsqueeze(-1)
        else:
            taus = taus.reshape(batch_size, num_tau, 1).to(self.pis.device, torch.float32)
        taus = taus * cvar
        cos = torch.cos(taus * self.pis)
        return cos, taus

    def observation_processor(self, x, num_tau=8, cvar=1.0, taus=None):
        features = encode_observation(self.self_encoder, self.object_encoder, x, self.max_object_num,
                                      self.object_dimension, self.object_feature_dimension)
        batch_size = features.shape[0]
        cos, taus = self.calc_cos(batch_size, num_tau, cvar, taus)
        cos = cos.view(batch_size * num_tau, self.n)
        cos_features = relu(self.cos_embedding(cos)).view(batch_size, num_tau, self.concat_feature_dimension)
        features = (features.unsqueeze(1) * cos_features).view(batch_size * num_tau, self.concat_feature_dimension)
        return features, taus

    def forward(self, x, actions, num_tau=8, cvar=1.0, taus=None):
        batch_size = x[0].shape[0]
        features, taus = self.observation_processor(x, num_tau, cvar, taus)
        features = relu(self.hidden_layer(features))
        action_features = self.action_encoder(actions)
        features = features.view(batch_size, num_tau, self.hidden_dimension)
        features = (action_features.unsqueeze(1) * features).view(batch_size * num_tau, self.hidden_dimension)
        features = relu(self.hidden_layer_2(features))
        quantiles = self.output_layer(features)
        return quantiles.view(batch_size, num_tau), taus

    def get_constructor_parameters(self):
        return dict(self_dimension=self.self_dimension, object_dimension=self.object_dimension,
                    max_object_num=self.max_object_num, self_feature_dimension=self.self_feature_dimension,
                    object_feature_dimension=self.object_feature_dimension,
                    concat_feature_dimension=self.concat_feature_dimension, hidden_dimension=self.hidden_dimension,
                    action_dimension=self.action_dimension, seed=self.seed_id)
