#!/usr/bin/env python3
"""Bit-identity check of fused-critic / fused-IQN variants: run the critic update (AC-IQN, and the IQN update with
--iqn) at the bench shape on a fixed batch with the library ASVRL_LIB names, and save every reduced gradient and
the loss to an npz; --compare A B reports whether two dumps are bit-identical.

    ASVRL_LIB=variants/libasvrl_x.so python tools/fused_dump.py out_x.npz
    python tools/fused_dump.py --compare out_default.npz out_x.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(path, B=4096, N=32):
    import torch
    from tests.test_critic_fused_gpu import _batch, _critic_grads
    rows, _ = _batch(B, 11)
    g = torch.Generator(device="cuda").manual_seed(12)
    taus = torch.rand(2, B, N, generator=g, device="cuda")
    out = {}
    for enc in (False, True):
        grads, loss = _critic_grads("bf16", B, N, True, rows, taus, enc=enc)[:2]
        for k, v in grads.items():
            out[f"acq{int(enc)}/{k}"] = np.asarray(v, dtype=np.float32)
        out[f"acq{int(enc)}/loss"] = np.array([float(loss)], np.float32)
    from tests.test_iqn_fused_gpu import _batch as iqn_batch, _iqn_grads
    gi, li = _iqn_grads("bf16", B, N, True, iqn_batch(B, 13), taus)
    for k, v in gi.items():
        out[f"iqn/{k}"] = np.asarray(v, dtype=np.float32)
    out["iqn/loss"] = np.array([float(li)], np.float32)
    np.savez(path, **out)
    print("dumped", len(out), "arrays to", path)


def compare(a, b):
    za, zb = np.load(a), np.load(b)
    bad = [k for k in za.files if k not in zb.files or not np.array_equal(za[k], zb[k])]
    for k in bad[:20]:
        d = np.abs(za[k] - zb[k]).max() if k in zb.files else None
        print("DIFF", k, d)
    print("bit-identical" if not bad else f"{len(bad)} of {len(za.files)} arrays differ")
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    dump(sys.argv[1])
