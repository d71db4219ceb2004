#!/usr/bin/env python3
"""A/B of the AC-IQN critic update kernels (asvrl_critic_fused_variant: 8 = two waves per SIMD, 4 = one) at the
bench shape: the launch the learner issues (asvrl_critic_train_fused_tq, encoders in the launch) and the update
alone (asvrl_critic_train_fused), HIP events around `--launches` back-to-back launches, alternating the variants
`--reps` times; prints the medians (us per launch) as one JSON line.

    python tools/ab_fused_variant.py [--B 4096] [--launches 20] [--reps 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="8,4")
    ap.add_argument("--forms", default="tq,update")
    a = ap.parse_args()
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_critic import PartialArena, critic_train_fused, fused_variant
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState, target_q
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    from tests.test_critic_fused_gpu import _batch
    B, N = a.B, 32
    rows, _ = _batch(B, 3)
    taus = torch.rand(2, B, N, generator=torch.Generator(device="cuda").manual_seed(4), device="cuda")
    ag = Agent(seed=100, agent_type="AC-IQN")
    FusedAdam(ag.policy_local.actor.parameters(), lr=1e-4)
    FusedAdam(ag.policy_local.critic.parameters(), lr=1e-4)
    st = FusedACIQNState(ag.policy_local, ag.policy_target, B, N)
    target_q(st, rows, taus[0], st.q_next, st.na)
    arena = PartialArena(32 << 20, "cuda")
    critic = ag.policy_local.critic

    def one(tq):
        critic_train_fused(st.local_trunk, critic, taus[1], N, st.q_next.view(B, N), rows[:, 82], rows[:, 83], 0.99,
                           rows[:, 0:40], rows[:, 80:82], arena, tile_loss=st.tile_loss[0], encoders=True,
                           target=(st.target_trunk, taus[0], rows[:, 40:80], st.na) if tq else None)
        arena.segs, arena.off = [], 0

    res = {}
    stream = torch.cuda.current_stream()
    for rep in range(a.reps):
        for v in [int(x) for x in a.variants.split(",")]:
            for tq in [f == "tq" for f in a.forms.split(",")]:
                with fused_variant(v):
                    for _ in range(3):
                        one(tq)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(a.launches):
                        one(tq)
                    e1.record(stream)
                    torch.cuda.synchronize()
                res.setdefault(f"v{v}_{'tq' if tq else 'update'}", []).append(1e3 * e0.elapsed_time(e1) / a.launches)
    out = {k: {"median_us": sorted(x)[len(x) // 2], "all_us": [round(y, 2) for y in x]} for k, x in res.items()}
    out["B"] = B
    print(json.dumps(out))


if __name__ == "__main__":
    main()
