"""GPU: VecTrainer's dependency-chained graph schedule (two iterations per captured graph, the rollout
and learner streams ordered by the exact dependencies: act after the previous learn, learn after the
ring snapshot behind the previous push, weight updates after this iteration's act) against the
joined schedule (a full join of the two streams per iteration): the same operations on the same data,
so weights, losses, env state and replay state agree bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(agent_type, chain, iters):
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    tr = VecTrainer(n_envs=256, agent_type=agent_type, batch_size=256, num_tau=32, seed=21, graphs=True,
                    unroll=2, chain=chain, buffer_size=256 * 5 * 40, learning_starts=512)
    while tr.replay_size_host() < tr.learning_starts:
        tr.iteration()
    for _ in range(iters):
        out = tr.iteration()
    torch.cuda.synchronize()
    nets = [tr.local.actor, tr.local.critic] if agent_type == "AC-IQN" else [tr.local]
    params = torch.cat([p.detach().reshape(-1).float() for n in nets for p in n.parameters()])
    losses = torch.stack([torch.as_tensor(x, device="cuda").float().reshape(()) for x in out[:2]])
    return tr, params, losses


@pytest.mark.parametrize("agent_type", ["AC-IQN", "IQN"])
def test_chained_schedule_matches_joined(agent_type):
    a, pa, la = _run(agent_type, True, 8)
    b, pb, lb = _run(agent_type, False, 8)
    assert a._chained() and not b._chained()
    assert torch.isfinite(la).all()
    assert torch.equal(la, lb), (la, lb)
    assert torch.equal(pa, pb), float((pa - pb).abs().max())
    assert torch.equal(a.env.batch.rs, b.env.batch.rs)
    assert torch.equal(a.replay.state, b.replay.state)
    assert torch.equal(a.replay.ring, b.replay.ring)
