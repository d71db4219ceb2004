"""GPU: VecTrainer's dependency-chained graph schedule (the rollout and learner streams ordered by the
exact dependencies: act after the previous learn, learn after the ring snapshot behind the previous
push, weight updates after this iteration's act) against the joined schedule (a full join of the two
streams per iteration): the same operations on the same data, so weights, losses, env state and replay
state agree bit for bit. Two iterations per graph at 256 envs, and the bench's shape: ten iterations per
graph at 4096 envs, B = 4096, N = 32 -- after 40 pool streams were handed out in this process, the
state in which round 2's captured graphs met aliased streams (streams.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(agent_type, chain, iters, n_envs=256, batch=256, unroll=2, target_after_env=False, push_after_actor=None):
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    tr = VecTrainer(n_envs=n_envs, agent_type=agent_type, batch_size=batch, num_tau=32, seed=21, graphs=True,
                    unroll=unroll, chain=chain, buffer_size=max(n_envs * 5 * 40, 4 * n_envs * 5),
                    learning_starts=2 * batch, target_after_env=target_after_env,
                    push_after_actor=push_after_actor)
    while tr.replay_size_host() < tr.learning_starts:
        tr.iteration()
    for _ in range(iters):
        out = tr.iteration()
    torch.cuda.synchronize()
    nets = [tr.local.actor, tr.local.critic] if agent_type == "AC-IQN" else [tr.local]
    params = torch.cat([p.detach().reshape(-1).float() for n in nets for p in n.parameters()])
    losses = torch.stack([torch.as_tensor(x, device="cuda").float().reshape(()) for x in out[:2]])
    return tr, params, losses


def _same(a, pa, la, b, pb, lb):
    assert a._chained() and not b._chained()
    assert torch.isfinite(la).all()
    assert torch.equal(la, lb), (la, lb)
    assert torch.equal(pa, pb), float((pa - pb).abs().max())
    assert torch.equal(a.env.batch.rs, b.env.batch.rs)
    assert torch.equal(a.replay.state, b.replay.state)
    assert torch.equal(a.replay.ring, b.replay.ring)


@pytest.mark.parametrize("agent_type", ["AC-IQN", "IQN"])
def test_chained_schedule_matches_joined(agent_type):
    a, pa, la = _run(agent_type, True, 8)
    assert a.push_after_actor == (agent_type == "AC-IQN")
    b, pb, lb = _run(agent_type, False, 8)
    _same(a, pa, la, b, pb, lb)


def test_chained_schedule_target_after_env_matches_joined():
    """The schedule knob that holds the learner's target critic behind the same iteration's env step: an
    ordering only, so bit-identical to the joined schedule too."""
    a, pa, la = _run("AC-IQN", True, 8, target_after_env=True)
    b, pb, lb = _run("AC-IQN", False, 8)
    _same(a, pa, la, b, pb, lb)


def test_chained_schedule_push_beside_actor_matches_joined():
    """push_after_actor (on by default in the chained AC-IQN graph: the replay push and the reset behind it
    wait for the learner's ACTOR pass) switched off -- the push beside the ACTOR pass, round 5's earlier
    schedule: bit-identical to the joined schedule as well."""
    a, pa, la = _run("AC-IQN", True, 8, push_after_actor=False)
    assert not a.push_after_actor
    b, pb, lb = _run("AC-IQN", False, 8)
    assert not b.push_after_actor   # the joined schedule resolves the default to off
    _same(a, pa, la, b, pb, lb)


def test_push_after_actor_default_and_refusal():
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    tr = VecTrainer(n_envs=64, agent_type="AC-IQN", batch_size=64, num_tau=32, seed=1, chain=True, graphs=True, unroll=2)
    assert tr.push_after_actor
    for kw in (dict(chain=False, graphs=True, unroll=2), dict(chain=True, graphs=False, unroll=2)):
        with pytest.raises(ValueError, match="push_after_actor"):
            VecTrainer(n_envs=64, agent_type="AC-IQN", batch_size=64, num_tau=32, seed=1, push_after_actor=True, **kw)


def test_target_after_env_refused_where_it_would_be_ignored():
    """The knob orders two nodes of the chained graph: on the joined schedule or without graphs it would do
    nothing, so the constructor refuses it instead of letting a bench config record it."""
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    for kw in (dict(chain=False, graphs=True, unroll=2), dict(chain=True, graphs=False, unroll=2)):
        with pytest.raises(ValueError, match="target_after_env"):
            VecTrainer(n_envs=64, agent_type="AC-IQN", batch_size=64, num_tau=32, seed=1, target_after_env=True, **kw)


def test_chained_schedule_bench_shape_after_pool_wrap():
    from distributional_rl_decision_and_control_amd import streams
    pool = [torch.cuda.Stream() for _ in range(40)]   # torch's pool (32 per device) wraps around
    a, pa, la = _run("AC-IQN", True, 20, n_envs=4096, batch=4096, unroll=10)
    handles = [streams.capture_stream(a.device).cuda_stream, a.roll_stream().cuda_stream,
               streams.stream(a.device, "warmup").cuda_stream]
    assert len(set(handles)) == len(handles), "the schedule's streams must be distinct"
    assert not set(handles) & {s.cuda_stream for s in pool}, "a schedule stream is also a torch pool stream"
    del a
    b, pb, lb = _run("AC-IQN", False, 20, n_envs=4096, batch=4096, unroll=10)
    assert b.unroll == 10
    # a was deleted (its graph destroyed) before b captured: compare the numbers only
    assert torch.isfinite(la).all()
    assert torch.equal(la, lb), (la, lb)
    assert torch.equal(pa, pb), float((pa - pb).abs().max())


def test_target_critic_in_fused_launch_matches_separate(monkeypatch):
    """fused_update.TARGET_IN_FUSED (ABI 20): the loop with the target critic's forward inside the fused
    critic launch against the same loop with the separate asvrl_critic_forward launch -- the same values in
    the same order, so the chained loop's weights, losses, env and replay state agree bit for bit."""
    from distributional_rl_decision_and_control_amd import fused_update
    monkeypatch.setattr(fused_update, "TARGET_IN_FUSED", True)
    a, pa, la = _run("AC-IQN", True, 8)
    monkeypatch.setattr(fused_update, "TARGET_IN_FUSED", False)
    b, pb, lb = _run("AC-IQN", True, 8)
    assert torch.isfinite(la).all()
    assert torch.equal(la, lb), (la, lb)
    assert torch.equal(pa, pb), float((pa - pb).abs().max())
    assert torch.equal(a.env.batch.rs, b.env.batch.rs)
    assert torch.equal(a.replay.ring, b.replay.ring)

