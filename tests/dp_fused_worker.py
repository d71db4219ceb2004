"""Worker of tests/test_dp_fused_gpu.py (not a test module): the fused learner updates of one
rank on its share of a fixed batch, with the gradient all-reduce of fused_update._reduce_and_step's
data-parallel branch (asvrl_partial_sums -> GradSync -> FusedAdam.step_synced: asvrl_partial_sums_norm over the
averaged gradient, then asvrl_adam_step_pack writing the weight images; Rainbow: asvrl_adam_clip + re-pack).

    python tests/dp_fused_worker.py RANK WORLD PORT OUT.npz

world == 1 in the test process itself (sync=None: the single-GPU fused optimiser path, with the
gradient norm formed inside the reduction launch). Every rank builds identical networks and draws
the same batches from a CPU generator, then takes rows [rank * B / world, (rank + 1) * B / world).
"""
import copy
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

B_FULL, N, STEPS = 128, 32, 2


def _rows(B, seed, discrete):
    g = torch.Generator().manual_seed(seed)
    rows = torch.zeros(B, 88)
    for c in (0, 40):
        rows[:, c:c + 7] = torch.randn(B, 7, generator=g) * 3
        rows[:, c + 7:c + 32] = torch.randn(B, 25, generator=g) * 3
        rows[:, c + 32:c + 37] = (torch.rand(B, 5, generator=g) > 0.4).float()
    if discrete:
        rows[:, 80] = torch.randint(0, 25, (B,), generator=g).float()
    else:
        rows[:, 80:82] = torch.rand(B, 2, generator=g) * 2 - 1
    rows[:, 82] = torch.randn(B, generator=g)
    rows[:, 83] = (torch.rand(B, generator=g) > 0.8).float()
    rows[:, 84] = torch.rand(B, generator=g) * 0.9 + 0.1   # Rainbow: IS weight column (PER rows)
    return rows


def _taus(k, B, seed):
    return torch.rand(k, B, N, generator=torch.Generator().manual_seed(seed))


def run(agent, rank, world, sync):
    """STEPS updates of `agent` on this rank's rows; returns dict of numpy arrays."""
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    dev = torch.device("cuda", 0)
    Bw = B_FULL // world
    sl = slice(rank * Bw, (rank + 1) * Bw)
    out = {}
    if agent == "AC-IQN":
        from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState, ac_iqn_update_fused2
        from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import AC_IQN_Policy
        mk = lambda: AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1, 1], [-1, 1]], device=dev,  # noqa
                                   seed=100)
        loc, tgt = mk(), mk()
        ao, co = FusedAdam(loc.actor.parameters(), lr=1e-4), FusedAdam(loc.critic.parameters(), lr=1e-4)
        st = FusedACIQNState(loc, tgt, Bw, N)
        for k in range(STEPS):
            rows = _rows(B_FULL, 10 + k, False)[sl].contiguous().to(dev)
            taus = _taus(3, B_FULL, 20 + k)[:, sl].contiguous().to(dev)
            cl, al, cg, ag = ac_iqn_update_fused2(st, loc, ao, co, co.grads, ao.grads, rows, taus=taus, sync=sync)
            torch.cuda.synchronize()
            out[f"loss{k}"] = np.array([cl.item(), al.item()])
            out[f"critic_grad{k}"] = co.grads.flat.cpu().numpy()
            out[f"actor_grad{k}"] = ao.grads.flat.cpu().numpy()
            out[f"params{k}"] = np.concatenate([co.flat.cpu().numpy(), ao.flat.cpu().numpy()])
    elif agent == "IQN":
        from distributional_rl_decision_and_control_amd.fused_iqn import FusedIQNState, iqn_update_fused
        from distributional_rl_decision_and_control_amd.policy.IQN_model import IQN_Policy
        loc = IQN_Policy(**DEFAULT_NET, action_size=25, device=dev, seed=3).to(dev)
        tgt = IQN_Policy(**DEFAULT_NET, action_size=25, device=dev, seed=3).to(dev)
        opt = FusedAdam(loc.parameters(), lr=1e-4)
        st = FusedIQNState(loc, tgt, Bw, N)
        for k in range(STEPS):
            rows = _rows(B_FULL, 30 + k, True)[sl].contiguous().to(dev)
            taus = _taus(2, B_FULL, 40 + k)[:, sl].contiguous().to(dev)
            loss, gn = iqn_update_fused(st, loc, opt, opt.grads, rows, taus=taus, sync=sync)
            torch.cuda.synchronize()
            out[f"loss{k}"] = np.array([loss.item()])
            out[f"grad{k}"] = opt.grads.flat.cpu().numpy()
            out[f"params{k}"] = opt.flat.cpu().numpy()
    else:   # Rainbow (fused_rainbow.FusedRainbow.update: one all-reduce)
        from distributional_rl_decision_and_control_amd.fused_rainbow import FusedRainbow
        from distributional_rl_decision_and_control_amd.policy.Rainbow_model import Rainbow_Policy
        loc = Rainbow_Policy(**DEFAULT_NET, action_size=25, atoms=51, device=dev, seed=9).to(dev)
        tgt = copy.deepcopy(loc)
        for p in tgt.parameters():
            p.requires_grad_(False)
        opt = FusedAdam(loc.parameters(), lr=1e-4)
        sup = torch.linspace(-1.0, 1.0, 51, device=dev)
        fr = FusedRainbow(loc, tgt, Bw, sup)
        ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        for k in range(STEPS):
            rows = _rows(B_FULL, 50 + k, True)[sl].contiguous().to(dev)
            loss, gn = fr.update(opt, opt.grads, rows, seed=11, counter_dev=ctr, sync=sync)
            ctr += 1
            torch.cuda.synchronize()
            # per-sample losses of this rank's rows; the mean over ranks is the full-batch loss
            out[f"loss{k}"] = loss.cpu().numpy()
            out[f"grad{k}"] = opt.grads.flat.cpu().numpy()
            out[f"params{k}"] = opt.flat.cpu().numpy()
    return out


def main():
    rank, world, port, path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributional_rl_decision_and_control_amd.learner import GradSync
    sync = GradSync()
    assert sync.world == world and not sync.avg_supported   # gloo: staged through host memory
    res = {}
    for agent in ("AC-IQN", "IQN", "Rainbow"):
        for k, v in run(agent, rank, world, sync).items():
            res[f"{agent}/{k}"] = v
    np.savez(path, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
