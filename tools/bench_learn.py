#!/usr/bin/env python3
"""The AC-IQN learner alone (ac_iqn_update_fused2 at the bench shape, B = 4096, N = 32, random replay rows):
ms per update from HIP events over `--steps` eager updates after a warm-up, three times. Run it under
rocprofv3 --kernel-trace --stats for per-kernel times.

    python tools/bench_learn.py [--steps 30] [--B 4096]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--N", type=int, default=32)
    a = ap.parse_args()
    from distributional_rl_decision_and_control_amd import fused_update as fu
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import AC_IQN_Policy
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    B, N = a.B, a.N
    loc, tgt = [AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1, 1], [-1, 1]], device="cuda", seed=100)
                for _ in range(2)]
    fao, fco = FusedAdam(loc.actor.parameters(), lr=1e-4), FusedAdam(loc.critic.parameters(), lr=1e-4)
    st = fu.FusedACIQNState(loc, tgt, B, N)
    g = torch.Generator(device="cuda").manual_seed(1)
    rows = torch.zeros(B, 88, device="cuda")
    for c in (0, 40):
        rows[:, c:c + 32] = torch.randn(B, 32, generator=g, device="cuda") * 3
        rows[:, c + 32:c + 37] = (torch.rand(B, 5, generator=g, device="cuda") > 0.3).float()
    rows[:, 80:82] = torch.rand(B, 2, generator=g, device="cuda") * 2 - 1
    rows[:, 82] = torch.randn(B, generator=g, device="cuda")
    rows[:, 83] = (torch.rand(B, generator=g, device="cuda") > 0.9).float()
    taus = torch.rand(3, B, N, generator=g, device="cuda")
    for rep in range(3):
        for _ in range(5):
            fu.ac_iqn_update_fused2(st, loc, fao, fco, fco.grads, fao.grads, rows, taus=taus)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            fu.ac_iqn_update_fused2(st, loc, fao, fco, fco.grads, fao.grads, rows, taus=taus)
        e1.record()
        torch.cuda.synchronize()
        print(f"run {rep}: {e0.elapsed_time(e1) / a.steps:.4f} ms per update", flush=True)


if __name__ == "__main__":
    main()
