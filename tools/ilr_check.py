#!/usr/bin/env python3
"""VERDICT r04 item 2 measured: the fused critic update with its three trunk layers' partials reduced
inside the launch by a last arriver per 1 KB tile (variant build -DASVRL_INLAUNCH_REDUCE, never shipped).
Runs one update through the normal path (the launch, then partial_sums) and compares the in-launch sums
with partial_sums' gradients, reports how the 258 tiles were spread over the 256 workgroups, and times
the launch (tools/fused_time.py does the timing of both builds).

    ASVRL_LIB=variants/libasvrl_ilr.so python tools/ilr_check.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from distributional_rl_decision_and_control_amd import _abi
    from tests.test_critic_fused_gpu import _batch, _critic_grads
    B, N = 4096, 32
    rows, _ = _batch(B, 11)
    g = torch.Generator(device="cuda").manual_seed(12)
    taus = torch.rand(2, B, N, generator=g, device="cuda")
    grads, _ = _critic_grads("bf16", B, N, True, rows, taus, enc=True)
    n = (128 * 128 + 128) + (128 * 256 + 128) + (256 * 64 + 256)
    out = np.zeros(n, np.float32)
    won = np.zeros(1024, np.uint32)
    L = _abi.lib()
    fn = L.asvrl_debug_inlaunch_reduce
    fn.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]
    assert fn(out.ctypes.data, n, won.ctypes.data, 1024) == 0
    ref = np.concatenate([grads["hidden_layer_2.weight"].ravel(), grads["hidden_layer_2.bias"],
                          grads["hidden_layer.weight"].ravel(), grads["hidden_layer.bias"],
                          grads["cos_embedding.weight"].ravel(), grads["cos_embedding.bias"]])
    rel = np.abs(out - ref).max() / np.abs(ref).max()
    w = won[:256]
    print(json.dumps({"max_rel_diff_vs_partial_sums": float(rel), "tiles": int(w.sum()),
                      "workgroups_that_reduced": int((w > 0).sum()), "max_tiles_one_workgroup": int(w.max()),
                      "tiles_of_top4": [int(x) for x in np.sort(w)[::-1][:4]]}))


if __name__ == "__main__":
    main()
