#!/usr/bin/env python3
"""Per-phase timing of asvrl_critic_train_fused from s_memtime stamps (variant build:
python tools/build_variant.py stamps asvrl_critic_fused.hip=-DASVRL_FUSED_STAMPS), at the bench shape.
Prints, per phase, the mean cycles from the previous barrier's release to this barrier's arrival
(compute) and from arrival to release (wait), over every wave of every workgroup and the first 8 rounds.

    ASVRL_LIB=variants/libasvrl_stamps.so python tools/fused_stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["stage", "L0", "L1", "L2", "loss", "dz2", "dW2+L3", "dW1+L4+dWc"]


def main():
    from distributional_rl_decision_and_control_amd import _abi
    from tests.test_critic_fused_gpu import _batch, _critic_grads
    B, N = 4096, 32
    rows, _ = _batch(B, 3)
    taus = torch.rand(2, B, N, device="cuda")
    for _ in range(3):
        _critic_grads("bf16", B, N, True, rows, taus)
    torch.cuda.synchronize()
    L = _abi.lib()
    n = 1024 * 4 * 8 * 32
    buf = (C.c_uint64 * n)()
    L.asvrl_debug_fused_stamps.argtypes = [C.c_void_p, C.c_int64]
    assert L.asvrl_debug_fused_stamps(buf, n) == 0
    allst = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 4, 8, 32).astype(np.float64)
    groups = int(L.asvrl_critic_fused_groups(B, N))
    allst = allst[:groups]
    st = allst[..., :16]
    arr, rel = st[..., 0::2], st[..., 1::2]          # arrival / release at barrier k
    prev_rel = np.concatenate([np.roll(rel[..., -1:], 1, axis=2), rel[..., :-1]], axis=-1)
    comp = arr - prev_rel
    wait = rel - arr
    comp, wait = comp[:, :, 1:], wait[:, :, 1:]       # round 0's stage phase has no previous release
    tot = 0.0
    for k, ph in enumerate(PHASES):
        c, w = comp[..., k].mean(), wait[..., k].mean()
        tot += c + w
        print(f"{ph:12s} compute {c:8.0f}  wait {w:8.0f}  (max wait {wait[..., k].max():8.0f})")
    print(f"per round {tot:.0f} cycles; rounds per workgroup {8}, groups {groups}")
    # marks inside phases (slot, the barrier release the phase starts from): cycles since that release
    marks = [(16, 1, "L0: first cos block done"), (17, 3, "L1: MFMAs issued+landed"), (18, 5, "L2: MFMAs done"),
             (31, 7, "loss: computed"), (19, 11, "dW2 grid done"), (20, 11, "L3 MFMAs done"),
             (21, 11, "L3 epilogue (dz1) done"), (22, 13, "dW1 grid done"), (23, 13, "next-round stage done"),
             (24, 13, "L4 blk0 MFMAs done"), (25, 13, "L4 blk0 epilogue done"), (26, 13, "L4 blk0 dF sums done"),
             (27, 13, "L4 blk1 MFMAs done"), (28, 13, "L4 blk1 epilogue done"), (29, 13, "L4 blk1 dF sums done"),
             (30, 13, "encoder sums done"), (14, 13, "dWc done (phase end)")]
    rounds = allst[:, :, 1:]
    for slot, start, label in marks:
        d = rounds[..., slot] - rounds[..., start]
        print(f"  mark {slot:2d} {label:28s} {d.mean():8.0f}")


if __name__ == "__main__":
    main()
