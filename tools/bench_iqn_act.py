#!/usr/bin/env python3
"""act_iqn alone: the IQN_ACT critic launch over N robot rows (K = 32 taus each), HIP-event timed.
    python tools/bench_iqn_act.py [--rows 20480] [--iters 50]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20480)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_iqn import IqnPack, iqn_act
    ag = Agent(seed=1, agent_type="IQN")
    pack = IqnPack(ag.policy_local)
    g = torch.Generator(device="cuda").manual_seed(0)
    obs = torch.randn(a.rows, 40, device="cuda", generator=g)
    obs[:, 32:37] = (obs[:, 32:37] > 0).float()
    acts = torch.zeros(a.rows, 2, dtype=torch.float64, device="cuda")
    step = torch.zeros(1, dtype=torch.int64, device="cuda")
    for _ in range(5):
        iqn_act(pack, None, acts, step, 1, 1e6, 0.25, 0.6, 0.05, 3, obs=obs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        iqn_act(pack, None, acts, step, 1, 1e6, 0.25, 0.6, 0.05, 3, obs=obs)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    flops = 2.0 * a.rows * 32 * (64 * 256 + 256 * 128 + 128 * 128 + 128 * 32)
    print(f"iqn_act rows={a.rows}: {ms * 1e3:.1f} us/launch, {flops / ms / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
