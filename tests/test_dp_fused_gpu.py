"""GPU, 2 ranks on one GPU over gloo: the data-parallel branch of the FUSED learners.

fused_update._reduce_and_step's data-parallel branch is the multi-rank path of every hand-written update: the
weight-gradient partials are reduced (asvrl_partial_sums), all-reduced (GradSync), then the norm is formed over the
averaged gradient and clip + Adam write the weight images in one launch (FusedAdam.step_synced:
asvrl_partial_sums_norm + asvrl_adam_step_pack; Rainbow: asvrl_adam_clip and a re-pack). AC-IQN all-reduces the critic gradient,
steps the critic, then evaluates the actor loss through the UPDATED critic and all-reduces the
actor gradient (agent.py:395-427: two collectives); IQN (agent.py:466-472) and Rainbow
(agent.py:632-637) one each.

Two worker processes (tests/dp_fused_worker.py) each run two updates of all three agents on half
of a fixed batch (B = 128, N = 32); this process runs the same two updates on the full batch on one
rank (sync=None: the single-GPU fused path, norm inside the reduction). Checked:
  * both ranks end with bit-identical weights and gradients (a missing actor sync, a rank-local
    clip or a stale weight image diverges them),
  * the averaged gradients equal the full-batch gradients (rel. 1e-4 of the gradient norm: the
    per-row bf16 activations are identical, only f32 summation orders differ),
  * losses within 1e-5 rel., and weights after both steps within 1e-5 abs. (a tenth of one
    Adam step of lr = 1e-4: Adam's first steps are +-lr per element, so this catches clip-before-
    average, a skipped sync or a wrong actor/critic order, which move weights by O(lr)).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def ranks(tmp_path_factory):
    d = tmp_path_factory.mktemp("dp")
    port = str(_port())
    env = dict(os.environ, OMP_NUM_THREADS="2")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_fused_worker.py"), str(r), "2", port,
                               str(d / f"rank{r}.npz")], env=env) for r in range(2)]
    for p in procs:
        p.wait(timeout=240)
    assert all(p.returncode == 0 for p in procs), [p.returncode for p in procs]
    return [dict(np.load(d / f"rank{r}.npz")) for r in range(2)]


@pytest.fixture(scope="module")
def full():
    sys.path.insert(0, HERE)
    import dp_fused_worker as w
    return {a: w.run(a, 0, 1, None) for a in ("AC-IQN", "IQN", "Rainbow")}


def _grad_keys(agent):
    return ["critic_grad", "actor_grad"] if agent == "AC-IQN" else ["grad"]


@pytest.mark.parametrize("agent", ["AC-IQN", "IQN", "Rainbow"])
def test_fused_dp_two_ranks(ranks, full, agent):
    r0, r1 = ranks
    ref = full[agent]
    for k in range(2):
        for g in _grad_keys(agent) + ["params"]:
            key = f"{agent}/{g}{k}"
            assert np.array_equal(r0[key], r1[key]), f"ranks diverged: {key}"
        for g in _grad_keys(agent):
            got, want = r0[f"{agent}/{g}{k}"], ref[f"{g}{k}"]
            err = np.abs(got - want).max() / max(np.linalg.norm(want), 1e-30)
            assert err < 1e-4, (agent, g, k, err)
        if agent == "Rainbow":   # per-sample losses: the ranks hold the two halves of the batch
            got_l = np.concatenate([r0[f"{agent}/loss{k}"], r1[f"{agent}/loss{k}"]])
        else:                    # batch means: the full-batch loss is the mean of the two halves
            got_l = 0.5 * (r0[f"{agent}/loss{k}"] + r1[f"{agent}/loss{k}"])
        np.testing.assert_allclose(got_l, ref[f"loss{k}"], rtol=1e-5, atol=1e-7)
        dp = np.abs(r0[f"{agent}/params{k}"] - ref[f"params{k}"]).max()
        assert dp < 1e-5, (agent, k, dp)
