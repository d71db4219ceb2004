"""CPU, world_size 2 over gloo: the data-parallel learn step's gradient path.

Each rank holds half of a batch; FlatGrads + GradSync (the all-reduce used between backward
and clip in learner.py) must give every rank the gradient of the full-batch loss, so the
clipped Adam update is identical on both ranks and equal to the single-process update on the
concatenated batch (SURVEY.md 8e gradient-equivalence test, 1e-6 rel). The loss here is the
oracle's torch restatement of agent.py:406-412 (the HIP kernel needs a GPU)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import learn_ref as lr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(B=16, N=8):
    g = torch.Generator().manual_seed(0)
    s = (torch.randn(B, 7, generator=g), torch.randn(B, 5, 5, generator=g), (torch.rand(B, 5, generator=g) > 0.4).float())
    a = torch.rand(B, 2, generator=g) * 2 - 1
    qt = torch.randn(B, N, generator=g)
    taus = torch.rand(B, N, 1, generator=g)
    return s, a, qt, taus


def _critic():
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import Critic
    return Critic(7, 5, 5, 56, 40, 256, 128, 2, "cpu", 101)


def _step(critic, fg, sync, s, a, qt, taus):
    from distributional_rl_decision_and_control_amd.learner import _clip
    fg.zero_()
    qe, _ = critic(s, a, taus.shape[1], taus=taus)
    lr.quantile_huber(qt, qe, taus).backward()
    if sync is not None:
        sync(fg)
    _clip(fg.params, 0.5)
    return fg.flat.clone()


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributional_rl_decision_and_control_amd.learner import FlatGrads, GradSync
    critic = _critic()
    fg = FlatGrads(critic.parameters())
    opt = torch.optim.Adam(critic.parameters(), lr=1e-4)
    s, a, qt, taus = _data()
    h = qt.shape[0] // world
    sl = slice(rank * h, (rank + 1) * h)
    g = _step(critic, fg, GradSync(), tuple(x[sl] for x in s), a[sl], qt[sl], taus[sl])
    opt.step()
    w = torch.cat([p.detach().reshape(-1) for p in critic.parameters()])
    out[rank] = (g.numpy(), w.numpy())
    dist.destroy_process_group()


def test_two_rank_gradient_equals_full_batch():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    from distributional_rl_decision_and_control_amd.learner import FlatGrads
    critic = _critic()
    fg = FlatGrads(critic.parameters())
    opt = torch.optim.Adam(critic.parameters(), lr=1e-4)
    s, a, qt, taus = _data()
    g_full = _step(critic, fg, None, s, a, qt, taus).numpy()
    opt.step()
    w_full = torch.cat([p.detach().reshape(-1) for p in critic.parameters()]).numpy()
    g0, w0 = out[0]
    g1, w1 = out[1]
    np.testing.assert_array_equal(g0, g1)
    np.testing.assert_array_equal(w0, w1)
    np.testing.assert_allclose(g0, g_full, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(w0, w_full, rtol=1e-6, atol=1e-8)
