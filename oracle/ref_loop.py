"""The reference's training loop on the CPU, restated for the bench's reference-style baseline (TEST / BASELINE
INFRASTRUCTURE ONLY; only bench.py's cpu_baseline runs it, as child processes).

One process = one Trainer.learn (trainer.py:97-172) on one MarineNavEnv3 with an AC-IQN agent:
  per env step   every active vessel acts through the Actor on a batch of one (agent.py:207-225 act_ac_iqn,
                 epsilon-greedy at the schedule's final 0.05, trainer.py:257-264), env.step
                 (oracle/env_numpy.NpMarineEnv, pinned to the reference's traces), one replay add per vessel
                 (replay_buffer.py:22-24), the trainer's deactivation / episode end (trainer.py:157-172);
  every 4 steps  one train_AC_IQN at BATCH_SIZE = 64, N = N' = 8 (agent.py:386-432; oracle/learn_ref.ACIQNRef,
                 pinned to the reference's captured updates) once the buffer holds 64 transitions.
torch and numpy on one thread each (OMP_NUM_THREADS=1), like the reference's default single process.

    python -m oracle.ref_loop --seconds 8 --seed 0 [--env-only]   -> one JSON line {steps, seconds, learns}
"""
import argparse
import json
import os
import random
import sys
import time
import warnings
from collections import deque

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _state_rows(batch):
    """ReplayBuffer.state_batch (replay_buffer.py:51-69): (self, objects padded to 5, mask) as f32 tensors."""
    import torch
    B = len(batch)
    s = np.zeros((B, 7), np.float32)
    o = np.zeros((B, 5, 5), np.float32)
    m = np.zeros((B, 5), np.float32)
    for i, (own, objs) in enumerate(batch):
        s[i] = own
        for k, ob in enumerate(objs):
            o[i, k] = ob
            m[i, k] = 1.0
    return torch.from_numpy(s), torch.from_numpy(o), torch.from_numpy(m)


def train_loop(seconds, seed=0, env_only=False):
    import torch
    from oracle import env_numpy as en
    from oracle import learn_ref as lr
    torch.set_num_threads(1)
    warnings.simplefilter("ignore")
    g = torch.Generator().manual_seed(seed)

    def lin(fout, fin):   # nn.Linear's default init range
        b = 1.0 / np.sqrt(fin)
        return ((torch.rand(fout, fin, generator=g) * 2 - 1) * b).numpy(), ((torch.rand(fout, generator=g) * 2 - 1) * b).numpy()
    actor, critic = {}, {}
    for sd, layers in ((actor, [("self_encoder.0", 56, 7), ("object_encoder.0", 40, 5), ("hidden_layer", 128, 256),
                                ("hidden_layer_2", 128, 128), ("output_layer", 2, 128)]),
                       (critic, [("self_encoder.0", 56, 7), ("object_encoder.0", 40, 5), ("cos_embedding", 256, 64),
                                 ("action_encoder.0", 128, 2), ("hidden_layer", 128, 256), ("hidden_layer_2", 128, 128),
                                 ("output_layer", 1, 128)])):
        for name, fout, fin in layers:
            sd[name + ".weight"], sd[name + ".bias"] = lin(fout, fin)
    agent = lr.ACIQNRef(actor, critic)
    memory = deque(maxlen=1_000_000)
    rnd = random.Random(249)
    env = en.NpMarineEnv(seed=seed, num_robots=5, num_obs=4, min_start_goal_dis=40.0)
    obs, _, _ = env.reset()
    steps = learns = 0
    t0 = time.perf_counter()
    while True:
        eps = 0.05   # trainer.py:257-264 after its exploration fraction: the steady state's act cost
        acts = []
        for v, ob in zip(env.robots, obs):
            if v.deactivated:
                acts.append(None)
            elif env_only or rnd.random() <= eps:
                acts.append(np.random.uniform(-1.0, 1.0, 2))
            else:
                with torch.no_grad():
                    a = lr.actor_forward(agent.actor, _state_rows([ob]))
                acts.append(a[0].numpy().astype(np.float64))
        nxt, rew, done, _ = env.step(acts, True)
        steps += 1
        for i, v in enumerate(env.robots):
            if v.deactivated:
                continue
            memory.append((obs[i], acts[i], rew[i], nxt[i] if nxt[i][0] is not None else obs[i], done[i]))
            if v.collision or v.reach_goal:
                v.deactivated = True
        obs = nxt
        if not env_only and steps % 4 == 0 and len(memory) >= 64:
            batch = rnd.sample(memory, 64)
            s = _state_rows([b[0] for b in batch])
            ns = _state_rows([b[3] for b in batch])
            a = torch.tensor(np.array([b[1] for b in batch]), dtype=torch.float32)
            r = torch.tensor([[float(b[2])] for b in batch])
            d = torch.tensor([[float(b[4])] for b in batch])
            taus = [torch.rand(64, 8, 1) for _ in range(3)]
            agent.train(s, a, r, ns, d, taus)
            learns += 1
        if all(v.deactivated for v in env.robots) or env.episode_timesteps >= 1000:
            obs, _, _ = env.reset()
        if steps % 8 == 0 and time.perf_counter() - t0 >= seconds:
            return {"steps": steps, "seconds": time.perf_counter() - t0, "learns": learns}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--env-only", action="store_true")
    a = ap.parse_args()
    print(json.dumps(train_loop(a.seconds, a.seed, a.env_only)))


if __name__ == "__main__":
    main()
