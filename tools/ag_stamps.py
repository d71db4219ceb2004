#!/usr/bin/env python3
"""Per-phase timing of asvrl_actor_grads[_adam] from s_memrealtime stamps (variant build:
python tools/build_variant.py agstamps asvrl_wgrad.hip=-DASVRL_AG_STAMPS), at the bench shape (B = 4096).
For each workgroup role (tile split, tile finisher, encoder fold, output layer, loss) prints when its phase
points were reached, in us after the first workgroup started: median and max over the workgroups.
Stamps: 0 start, 1 operands staged + MFMAs done (output layer: its sums), 2 slab stored, 3 arrival
returned (finisher), 4 slabs merged, 5 gradients and norm partial written. (Rows 6-10 were the in-launch
optimiser's phases, removed: profiles/r03p1_fused_adam_timeout.txt.)

    ASVRL_LIB=variants/libasvrl_agstamps.so python tools/ag_stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.fused_mlp import MlpPack, actor_grads
    from tests.test_actor_grads_gpu import _setup
    adam = False
    B = 4096
    actor, opt, ab, ws = _setup("bf16", B, seed=3)
    pk = MlpPack(actor, "actor", "bf16")
    segs = pk.adam_segments(opt)
    L = _abi.lib()
    sp = (C.c_int32 * 2)()
    L.asvrl_debug_ag_split(B, sp)
    S, nch = sp[0], sp[1]
    nblk = 56 * S + 17
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(30):
        if it == 20:
            ev0.record()
        actor_grads(ws, ab, actor, step=opt.step_t)
    ev1.record()
    torch.cuda.synchronize()
    print(f"S={S} nch={nch} blocks={nblk} adam={adam}: {ev0.elapsed_time(ev1) / 10 * 1e3:.1f} us per launch "
          f"(events, back to back)")
    buf = (C.c_uint64 * (4096 * 12))()
    assert L.asvrl_debug_ag_stamps(buf, 4096 * 12) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 12)[:nblk].astype(np.int64)
    t0 = st[:, 0].min()
    us = (st - t0) / 100.0   # 100 MHz
    role = []
    for b in range(nblk):
        if b < 56 * S:
            role.append("tile")
        elif b < 56 * S + 16:
            role.append("out")
        else:
            role.append("loss")
    role = np.array(role)
    fin = st[:, 3] > 0   # tile splits that returned from the arrival as last (stamps are cleared at each start)
    for name, sel in [("tile split", role == "tile"), ("tile finisher", (role == "tile") & fin),
                      ("out split", role == "out"), ("loss", role == "loss")]:
        if not sel.any():
            continue
        row = []
        for k in range(6):
            v = us[sel, k]
            v = v[(v >= 0) & (v < 1e4)]
            row.append(f"{k}:{np.median(v):6.1f}/{v.max():6.1f}" if v.size else f"{k}:   -  ")
        print(f"{name:14s} n={int(sel.sum()):4d}  " + "  ".join(row))
    print("end of the last workgroup (max stamp):", f"{np.where(us < 1e4, us, 0).max():.1f} us")


if __name__ == "__main__":
    main()
