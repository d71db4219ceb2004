#!/usr/bin/env python3
"""Microbenchmark of the fused critic kernels at the bench shape (B=4096, N=N'=32): average
launch time of FWD / TRAIN / ACTOR with HIP events, plus the derived rates. Set ASVRL_LIB to
time an alternative build of libasvrl.so.

    python tools/bench_critic.py [--B 4096] [--N 32] [--iters 50]
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
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--act-rows", type=int, default=4096 * 5)
    a = ap.parse_args()
    from distributional_rl_decision_and_control_amd.fused_critic import (CriticPack, TrainBuffers, critic_actor_grad,
                                                                          critic_forward, critic_train)
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import Critic
    B, N = a.B, a.N
    torch.manual_seed(0)
    c = Critic(7, 5, 5, 56, 40, 256, 128, 2, "cuda", 101).cuda()
    pack = CriticPack(c)
    F = torch.rand(B, 256, device="cuda")
    G = torch.rand(B, 128, device="cuda")
    taus = torch.rand(B, N, device="cuda")
    qt = torch.randn(B, N, device="cuda")
    bufs = TrainBuffers(B, N, "cuda")
    q = torch.empty(B * N, device="cuda")
    dA = torch.empty(B, 2, device="cuda")
    dzF = torch.empty(B, 256, dtype=torch.bfloat16, device="cuda")
    dzG = torch.empty(B, 128, device="cuda")
    runs = {
        "fwd": lambda: critic_forward(pack, F, G, taus, N, q=q),
        "train": lambda: critic_train(pack, F, G, taus, qt, bufs, dzF=dzF, dzG=dzG, with_dFdG=False),
        "actor": lambda: critic_actor_grad(pack, F, G, taus, N, q, w_ae=c.action_encoder[0].weight, dA=dA),
    }
    # IQN modes at the same shape; act_iqn over the rollout's robot rows (4096 envs x 5)
    from distributional_rl_decision_and_control_amd.fused_iqn import IqnPack, iqn_act, iqn_forward_max, iqn_train
    from distributional_rl_decision_and_control_amd.policy.IQN_model import IQN_Policy
    inet = IQN_Policy(7, 5, 5, 56, 40, 256, 128, 25, "cuda", 101).cuda()
    ipack = IqnPack(inet)
    rows = torch.zeros(B, 88, device="cuda")
    rows[:, 80] = torch.randint(0, 25, (B,), device="cuda").float()
    rows[:, 82] = torch.randn(B, device="cuda")
    dz_out = torch.empty(B * N, 32, dtype=torch.bfloat16, device="cuda")
    n_act = a.act_rows
    F_act = torch.rand(n_act, 256, device="cuda")
    act64 = torch.zeros(n_act, 2, dtype=torch.float64, device="cuda")
    step = torch.zeros(1, dtype=torch.int64, device="cuda")
    runs.update({
        "iqn_max": lambda: iqn_forward_max(ipack, F, taus, N, q),
        "iqn_train": lambda: iqn_train(ipack, F, taus, bufs, dz_out, qt, rows[:, 80], rows[:, 82], rows[:, 83], 0.99,
                                       dzF),
        "iqn_act": lambda: iqn_act(ipack, F_act, act64, step, 1.0, 1e6, 0.25, 0.1, 0.1, 7),
    })
    out = {}
    for k, fn in runs.items():
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[k + "_us"] = 1e3 * e0.elapsed_time(e1) / a.iters
    R = B * N
    out["train_tflops"] = R * 229632 / (out["train_us"] * 1e-6) / 1e12
    out["lib"] = os.environ.get("ASVRL_LIB", "default")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
