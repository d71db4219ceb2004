"""GPU: the data-parallel learn path captured in a HIP graph with its RCCL all-reduces.

bench.py replays the whole rollout + learn iteration as one HIP graph at every world size on
RCCL, so the gradient all-reduces (GradSync, between the weight-gradient reduction and clip +
Adam, fused_update._reduce_and_step) are captured too. On one GPU this runs over a 1-rank RCCL
group with GradSync(force=True), which issues the same collectives a multi-rank run does (AVG over
one rank is the identity): capture must succeed, replays must stay finite and keep training."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rccl_group():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def _flat(tr):
    ps = list(tr.local.actor.parameters()) + list(tr.local.critic.parameters()) if tr.agent_type == "AC-IQN" \
        else list(tr.local.parameters())
    return torch.cat([p.detach().reshape(-1) for p in ps]).cpu().numpy()


@pytest.mark.parametrize("agent", ["AC-IQN", "IQN", "Rainbow"])
def test_graph_captured_allreduce(rccl_group, agent):
    from distributional_rl_decision_and_control_amd.learner import GradSync
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    sync = GradSync(force=True)
    assert sync.force and sync.avg_supported
    tr = VecTrainer(n_envs=256, agent_type=agent, batch_size=512 if agent != "Rainbow" else 256, num_tau=32,
                    seed=5, buffer_size=256 * 5 * 40, graphs=True, sync=sync)
    while tr.replay_size_host() < tr.learning_starts:
        tr.iteration()
    tr.iteration()
    assert tr.graphs and tr._graph is not None, "capture with the RCCL all-reduce failed"
    p0 = _flat(tr)
    losses = []
    for _ in range(6):
        out = tr.iteration()
        losses.append(float(out[0].item()))
    torch.cuda.synchronize()
    p1 = _flat(tr)
    assert np.all(np.isfinite(losses)) and np.all(np.isfinite(p1))
    assert not np.array_equal(p0, p1)
