#!/usr/bin/env python3
"""Per-phase timing of asvrl_learn_prologue from s_memrealtime stamps (variant build:
python tools/build_variant.py prostamps asvrl_mlp.hip=-DASVRL_PRO_STAMPS), at the bench shape (B = 4096,
N = 32, a 1e6-row ring). Stamps (each after draining the workgroup's outstanding memory operations):
0 start, 1 ring state + weight fragments arrived and the slot drawn, 2 the eight rows gathered,
3 taus and rows stored, LDS staged; inside the actor tile: 10 observation operands loaded, 11 first
encoder block done, 5 encoders done, 6 their barrier passed,
7 hidden layer done, 8 hidden layer 2 + output partials done, 9 its barrier passed; 4 the tile done. Prints median / max per half (the TRAIN
tiles on s, the target FWD tiles on s') in us after the first workgroup started.

    ASVRL_LIB=variants/libasvrl_prostamps.so python tools/prologue_stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributional_rl_decision_and_control_amd import _abi, learn_ops
    from distributional_rl_decision_and_control_amd.fused_update import FusedACIQNState, learn_prologue
    from distributional_rl_decision_and_control_amd.learner import FusedAdam
    from distributional_rl_decision_and_control_amd.policy.AC_IQN_model import AC_IQN_Policy
    from distributional_rl_decision_and_control_amd.vec_trainer import DEFAULT_NET
    B, N, cap = 4096, 32, 1_000_000
    loc, tgt = [AC_IQN_Policy(**DEFAULT_NET, value_ranges_of_action=[[-1, 1], [-1, 1]], device="cuda", seed=s)
                for s in (100, 7)]
    FusedAdam(loc.actor.parameters()), FusedAdam(loc.critic.parameters())
    st = FusedACIQNState(loc, tgt, B, N)
    ring = learn_ops.DeviceReplay(cap, device="cuda")
    ring.ring.normal_()
    ring.state[0], ring.state[1] = 12345, cap
    ctr = torch.tensor([17], dtype=torch.int64, device="cuda")
    taus = torch.empty(3, B, N, device="cuda")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(40):
        if it == 20:
            ev0.record()
        ctr += 1
        learn_prologue(st, ring, taus, 99, counter_dev=ctr)
    ev1.record()
    torch.cuda.synchronize()
    print(f"B={B}: {ev0.elapsed_time(ev1) / 20 * 1e3:.1f} us per prologue (+ counter increment), back to back")
    L = _abi.lib()
    T = B // 32
    nblk = 2 * T
    K = 12
    order = [0, 1, 2, 3, 10, 11, 5, 6, 7, 8, 9, 4]
    buf = (C.c_uint64 * (2048 * K))()
    assert L.asvrl_debug_pro_stamps(buf, 2048 * K) == 0
    s = np.frombuffer(buf, dtype=np.uint64).reshape(2048, K)[:nblk][:, order].astype(np.int64)
    us = (s - s[:, 0].min()) / 100.0
    for name, sel in [("train (s)", slice(0, T)), ("target (s')", slice(T, nblk))]:
        row = [f"{k}:{np.median(us[sel, c]):6.2f}/{us[sel, c].max():6.2f}" for c, k in enumerate(order)]
        print(f"{name:12s} " + "  ".join(row))
    d = np.diff(us, axis=1)
    print("median phase lengths (us):", " ".join(f"{order[c]}->{order[c + 1]}:{np.median(d[:, c]):.2f}"
                                                 for c in range(len(order) - 1)))
    print("start spread (us): median", f"{np.median(us[:, 0]):.2f}", "max", f"{us[:, 0].max():.2f}")
    print("end of the last workgroup:", f"{us[:, -1].max():.2f} us")


if __name__ == "__main__":
    main()
