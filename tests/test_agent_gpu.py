"""GPU parity of the drop-in Agent's distributional updates against the reference's own
train_AC_IQN / train_IQN / train_Rainbow outputs (tests/golden/learn_*.npz): same seeded
initial weights, the captured batch and tau draws injected, losses within 1e-5 relative
(fp32, GPU GEMM order vs CPU), weights after 1 and 3 Adam steps within 1e-4. AC-IQN and IQN
run both learners Agent.train can use: the hand-written kernels' f32 build (the default) and the
torch-autograd restatement."""
import numpy as np
import pytest
import torch

from oracle import env_oracle as eo

pytestmark = pytest.mark.gpu


def _batch(z, p, dev, long_actions=False):
    t = lambda k: torch.tensor(z[p + k], dtype=torch.float32, device=dev)  # noqa: E731
    s = (t("s_self"), t("s_obj"), t("s_mask"))
    ns = (t("ns_self"), t("ns_obj"), t("ns_mask"))
    a = t("a")
    a = a.long().view(-1, 1).float() if long_actions else a
    return s, a, t("r").unsqueeze(-1), ns, t("d").unsqueeze(-1)


def _cmp_sd(module, z, prefix):
    for k, v in module.state_dict().items():
        np.testing.assert_allclose(v.detach().cpu().numpy(), z[prefix + k], rtol=1e-4, atol=2e-6, err_msg=prefix + k)


def test_agent_init_matches_reference():
    from distributional_rl_decision_and_control_amd.agent import Agent
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    ag = Agent(seed=100, agent_type="AC-IQN")
    for k, v in ag.policy_local.actor.state_dict().items():
        np.testing.assert_array_equal(v.cpu().numpy(), z["init/actor/" + k])
    for k, v in ag.policy_target.critic.state_dict().items():
        np.testing.assert_array_equal(v.cpu().numpy(), z["init/critic/" + k])


@pytest.mark.parametrize("learner", ["fused-f32", "torch"])
def test_train_ac_iqn_matches_reference(learner):
    from distributional_rl_decision_and_control_amd.agent import Agent
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    ag = Agent(seed=100, agent_type="AC-IQN")
    ag.set_learner(learner)
    dev = ag.device
    for step in range(3):
        b = _batch(z, f"step{step}/", dev)
        ag.memory.sample = (lambda b=b: b)
        ag.tau_override = list(z[f"step{step}/taus"])
        cl, al = ag.train()
        np.testing.assert_allclose(cl, z[f"step{step}/critic_loss"], rtol=1e-5)
        np.testing.assert_allclose(al, z[f"step{step}/actor_loss"], rtol=1e-5)
        if step in (0, 2):
            _cmp_sd(ag.policy_local.actor, z, f"after{step}/actor/")
            _cmp_sd(ag.policy_local.critic, z, f"after{step}/critic/")


@pytest.mark.parametrize("learner", ["fused-f32", "torch"])
def test_train_ac_iqn_32_quantiles_matches_reference(learner):
    from distributional_rl_decision_and_control_amd.agent import Agent
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    ag = Agent(seed=100, agent_type="AC-IQN")
    ag.set_learner(learner)
    ag.num_tau = 32
    b = _batch(z, "n32/", ag.device)
    ag.memory.sample = (lambda: b)
    ag.tau_override = list(z["n32/taus"])
    cl, al = ag.train()
    np.testing.assert_allclose(cl, z["n32/critic_loss"], rtol=1e-5)
    np.testing.assert_allclose(al, z["n32/actor_loss"], rtol=1e-5)
    _cmp_sd(ag.policy_local.critic, z, "n32after/critic/")
    _cmp_sd(ag.policy_local.actor, z, "n32after/actor/")


def test_actor_forward_without_objects():
    """The x_2 is None path (AC_IQN_model.py:293-294)."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    z = np.load(eo.GOLDEN + "/learn_ac_iqn.npz")
    ag = Agent(seed=100, agent_type="AC-IQN")
    s = ag.state_to_tensor((z["fwd/noobj_self"].tolist(), [], []))
    assert s[1] is None
    with torch.no_grad():
        out = ag.policy_local.actor(s).cpu().numpy()
    np.testing.assert_allclose(out, z["fwd/noobj_actions"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("learner", ["fused-f32", "torch"])
def test_train_iqn_matches_reference(learner):
    from distributional_rl_decision_and_control_amd.agent import Agent
    z = np.load(eo.GOLDEN + "/learn_iqn.npz")
    ag = Agent(seed=100, agent_type="IQN")
    ag.set_learner(learner)
    for step in range(3):
        b = _batch(z, f"step{step}/", ag.device, long_actions=True)
        ag.memory.sample = (lambda b=b: b)
        ag.tau_override = list(z[f"step{step}/taus"])
        loss = ag.train()
        np.testing.assert_allclose(loss, z[f"step{step}/loss"], rtol=1e-5)
        if step in (0, 2):
            _cmp_sd(ag.policy_local, z, f"after{step}/")


def test_act_iqn_matches_reference():
    from distributional_rl_decision_and_control_amd.agent import Agent
    z = np.load(eo.GOLDEN + "/learn_iqn.npz")
    # act_iqn was captured after three train steps; rebuild that network
    ag = Agent(seed=100, agent_type="IQN")
    for k, v in ag.policy_local.state_dict().items():
        v.copy_(torch.tensor(z["after2/" + k]))
    st = (z["act/state_self"].tolist(), z["act/state_obj"].tolist())
    a, q, t = ag.act_iqn(st, eps=0.0, taus=torch.tensor(z["act/taus"]))
    assert a == int(z["act/action"])
    np.testing.assert_allclose(q, z["act/quantiles"], rtol=1e-4, atol=1e-5)


def test_train_rainbow_matches_reference():
    from distributional_rl_decision_and_control_amd.agent import Agent
    z = np.load(eo.GOLDEN + "/learn_rainbow.npz")
    d = [int(x) for x in z["dims"]]
    ag = Agent(seed=100, agent_type="Rainbow", self_feature_dimension=d[0], object_feature_dimension=d[1],
               concat_feature_dimension=d[2], hidden_dimension=d[3])
    # NoisyLinear's CPU init (sign * sqrt of randn) can differ in the last bit across host
    # ISAs; check it to a few ulp, then start both networks from the captured state exactly.
    for k, v in ag.policy_local.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), z["init/" + k], rtol=1e-6, atol=0)
        v.copy_(torch.tensor(z["init/" + k]))
    for k, v in ag.policy_target.state_dict().items():
        v.copy_(torch.tensor(z["init_target/" + k]))
    # the target noise the reference drew inside train (agent.py:612) is injected
    tsd = ag.policy_target.state_dict()
    for k in tsd:
        if "epsilon" in k:
            tsd[k].copy_(torch.tensor(z["b64/target_after/" + k]))
    dev = ag.device
    t = lambda k: torch.tensor(z["b64/" + k], device=dev)  # noqa: E731
    batch = (np.arange(64), (t("s_self"), t("s_obj"), t("s_mask")), t("actions").long(), t("returns"),
             (t("ns_self"), t("ns_obj"), t("ns_mask")), t("nonterminal"), t("weights"))
    ag.memory.sample = lambda bs: batch
    pr = []
    ag.memory.update_priorities = lambda i, p: pr.append(p)
    loss = ag.train_Rainbow(reset_target_noise=False)
    np.testing.assert_allclose(loss, z["b64/loss"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(pr[0], z["b64/loss"], rtol=1e-5, atol=1e-6)
    _cmp_sd(ag.policy_local, z, "after/")


def test_train_dqn_matches_reference():
    """train_DQN (agent.py:518-545), the BASELINE config 1 agent: two steps on the captured batches."""
    from distributional_rl_decision_and_control_amd.agent import Agent
    z = np.load(eo.GOLDEN + "/learn_dqn.npz")
    ag = Agent(seed=100, agent_type="DQN")
    for k, v in ag.policy_local.state_dict().items():
        np.testing.assert_array_equal(v.cpu().numpy(), z["init/" + k])
    for step in range(2):
        b = _batch(z, f"step{step}/", ag.device, long_actions=True)
        ag.memory.sample = (lambda b=b: b)
        loss = ag.train()
        np.testing.assert_allclose(loss, z[f"step{step}/loss"], rtol=1e-5)
    _cmp_sd(ag.policy_local, z, "after1/")
    st = (z["act/state_self"].tolist(), z["act/state_obj"].tolist())
    assert ag.act_dqn(st, eps=0.0) == int(z["act/action"])


@pytest.mark.parametrize("eps", [0.0, 0.5, 1.0])
def test_act_ac_iqn_robots_matches_per_robot_acts(eps):
    """Agent.act_ac_iqn_robots (the drop-in Trainer's per-step acts in one actor call) against one act_ac_iqn call
    per robot from the same random states: the same draws in the same order (python random and numpy), so the
    exploring robots' actions are identical and the greedy ones equal up to the batched GEMM's summation order;
    both generators end in the same state."""
    import random
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.envs.marinenav.env import MarineNavEnv3
    sched = {"timesteps": [0], "num_robots": [5], "num_cores": [0], "num_obstacles": [4], "min_start_goal_dis": [40.0]}
    env = MarineNavEnv3(seed=3, schedule=sched)
    states, _, _ = env.reset()
    ag = Agent(seed=100, agent_type="AC-IQN")
    random.seed(11)
    np.random.seed(12)
    per = [ag.act_ac_iqn(s, eps, use_eval=False) for s in states]
    r_after, n_after = random.random(), np.random.rand()
    random.seed(11)
    np.random.seed(12)
    bat = ag.act_ac_iqn_robots(states, eps, use_eval=False)
    assert (random.random(), np.random.rand()) == (r_after, n_after)
    assert len(bat) == len(per) == len(states)
    for a, b in zip(per, bat):
        np.testing.assert_allclose(np.asarray(b), np.asarray(a), rtol=1e-5, atol=1e-6)
