import sys, numpy as np, torch
sys.path.insert(0, '.')
from tests.test_critic_fused_gpu import _critic_grads, _reference_grads, _batch
for ops, B, N in [("f32", 128, 32), ("f32", 256, 32), ("f32", 256, 8), ("f32", 512, 16), ("f32", 64, 32)]:
    rows, _ = _batch(B, 5 + N)
    g = torch.Generator(device="cuda").manual_seed(7 + B)
    taus = torch.rand(2, B, N, generator=g, device="cuda")
    gf, lf = _critic_grads(ops, B, N, True, rows, taus)
    gu, lu = _critic_grads(ops, B, N, False, rows, taus)
    d = np.abs(gf["cos_embedding.weight"] - gu["cos_embedding.weight"])
    sc = np.abs(gu["cos_embedding.weight"]).max()
    bad = np.argwhere(d > 1e-4 * sc)
    rowsbad = sorted(set(bad[:, 0].tolist())); colsbad = sorted(set(bad[:, 1].tolist()))
    db = np.abs(gf["cos_embedding.bias"] - gu["cos_embedding.bias"]); 
    print(ops, B, N, "maxrel", d.max() / sc, "bad", len(bad), "rows", rowsbad[:40], len(rowsbad), "cols", colsbad[:20], len(colsbad), "biasbad", np.argwhere(db > 1e-4*np.abs(gu["cos_embedding.bias"]).max()).ravel()[:40].tolist(), flush=True)
