#!/usr/bin/env python3
"""Launch time of asvrl_critic_train_fused alone at the bench shape (B=4096, N=N'=32), HIP events
on its stream around `--iters` back-to-back launches, repeated `--reps` times (median reported).
Set ASVRL_LIB to time a variant build (tools/build_variant.py).

    ASVRL_LIB=variants/libasvrl_x.so python tools/fused_time.py [--iqn]
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
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--mode", default="fused", choices=["fused", "tq", "target"],
                    help="fused: the update launch; tq: the update with the target critic inside "
                         "(asvrl_critic_train_fused_tq); target: the separate target critic launch alone")
    a = ap.parse_args()
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_critic import critic_forward, critic_train_fused
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState, target_q
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    from tests.test_critic_fused_gpu import _batch
    B, N = a.B, a.N
    rows, _ = _batch(B, 3)
    taus = torch.rand(2, B, N, device="cuda")
    ag = Agent(seed=100, agent_type="AC-IQN")
    loc, tgt = ag.policy_local, ag.policy_target
    FusedAdam(loc.actor.parameters(), lr=1e-4)
    FusedAdam(loc.critic.parameters(), lr=1e-4)
    st = FusedACIQNState(loc, tgt, B, N)
    critic, arena = loc.critic, st.arena
    s_rows, a_rows, r_col, d_col = rows[:, 0:40], rows[:, 80:82], rows[:, 82], rows[:, 83]
    target_q(st, rows, taus[0], st.q_next, st.na)

    def launch():
        if a.mode == "target":
            critic_forward(st.target_trunk, None, None, taus[0], N, q=st.q_next, obs=rows[:, 40:80], act=st.na)
            return
        arena.off, arena.segs = 0, []
        critic_train_fused(st.local_trunk, critic, taus[1], N, st.q_next.view(B, N), r_col, d_col, 0.99, s_rows,
                           a_rows, arena, tile_loss=st.tile_loss[0], encoders=True,
                           target=(st.target_trunk, taus[0], rows[:, 40:80], st.na) if a.mode == "tq" else None)

    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    us = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            launch()
        e1.record()
        e1.synchronize()
        us.append(e0.elapsed_time(e1) * 1000.0 / a.iters)
    us.sort()
    print(json.dumps({"lib": os.environ.get("ASVRL_LIB", "default"), "mode": a.mode, "us_median": round(us[len(us) // 2], 2),
                      "us_min": round(us[0], 2), "us_all": [round(u, 1) for u in us]}))


if __name__ == "__main__":
    main()
