#!/usr/bin/env python3
"""Diagnostic (not a test): the per-workgroup weight-gradient partials of asvrl_critic_train_fused for kernel
variants 8 and 4 on one batch, compared workgroup by workgroup and layer by layer (which groups, which
rows / columns differ), and variant 8 run twice (determinism).

    python tools/debug_fused8.py [--B 4096]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    a = ap.parse_args()
    from distributional_rl_decision_and_control_amd.agent import Agent
    from distributional_rl_decision_and_control_amd.fused_critic import PartialArena, critic_train_fused, fused_variant
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState, target_q
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    from tests.test_critic_fused_gpu import _batch
    B, N = a.B, 32
    rows, _ = _batch(B, 31)
    taus = torch.rand(2, B, N, generator=torch.Generator(device="cuda").manual_seed(32), device="cuda")
    ag = Agent(seed=100, agent_type="AC-IQN")
    FusedAdam(ag.policy_local.actor.parameters(), lr=1e-4)
    FusedAdam(ag.policy_local.critic.parameters(), lr=1e-4)
    st = FusedACIQNState(ag.policy_local, ag.policy_target, B, N)
    target_q(st, rows, taus[0], st.q_next, st.na)
    critic = ag.policy_local.critic

    def run(v):
        arena = PartialArena(32 << 20, "cuda")
        arena.buf.fill_(float("nan"))
        with fused_variant(v):
            critic_train_fused(st.local_trunk, critic, taus[1], N, st.q_next.view(B, N), rows[:, 82], rows[:, 83],
                               0.99, rows[:, 0:40], rows[:, 80:82], arena, tile_loss=st.tile_loss[0], encoders=True)
        torch.cuda.synchronize()
        return arena.buf[:arena.off].cpu().numpy().copy()

    p8, p4, p8b = run(8), run(4), run(8)
    groups = int(st.local_trunk.L.asvrl_critic_fused_groups(B, N))
    out = {"B": B, "groups": groups, "v8_deterministic": bool(np.array_equal(p8, p8b, equal_nan=True))}
    if not out["v8_deterministic"]:
        d = np.abs(p8 - p8b)
        out["v8_rerun_max_diff"] = float(np.nanmax(d))
        out["v8_rerun_n_diff"] = int((d > 0).sum())
    layers = [("cos_emb", 256, 64), ("hidden", 128, 256), ("hidden2", 128, 128), ("out", 1, 128)]
    off = 0
    for name, M, K in layers:
        n = groups * (M * K + M)
        x8 = p8[off:off + n].reshape(groups, M * K + M)
        x4 = p4[off:off + n].reshape(groups, M * K + M)
        off += (n + 63) // 64 * 64
        scale = np.abs(x4).max() + 1e-30
        dg = np.abs(x8 - x4).max(axis=1) / scale
        worst = np.argsort(dg)[::-1][:8]
        rec = {"max": float(dg.max()), "groups_over_1e-4": int((dg > 1e-4).sum()),
               "worst_groups": [[int(g), float(dg[g])] for g in worst]}
        g = int(worst[0])
        w = np.abs(x8[g, :M * K] - x4[g, :M * K]).reshape(M, K) / scale
        rr, cc = np.unravel_index(np.argsort(w.reshape(-1))[::-1][:12], (M, K))
        rec["worst_elements_of_worst_group"] = [[int(r), int(c), float(w[r, c])] for r, c in zip(rr, cc)]
        rec["rows_over_1e-4"] = sorted(set(int(r) for r in np.nonzero(w > 1e-4)[0]))[:40]
        rec["cols_over_1e-4"] = sorted(set(int(c) for c in np.nonzero(w > 1e-4)[1]))[:40]
        rec["bias_err"] = float(np.abs(x8[g, M * K:] - x4[g, M * K:]).max() / scale)
        out[name] = rec
    print(json.dumps(out))


if __name__ == "__main__":
    main()
