#!/usr/bin/env python3
"""C51 projection kernel alone (asvrl_c51_project) at B in {64, 8192, 65536}: 50 launches per size in one
HIP graph timed with HIP events (also the workload for rocprofv3 --kernel-trace --stats); prints one line per size with
the bytes the projection moves (bench.c51_project_bytes) and the fraction of the HBM peak. ASVRL_LIB picks
a variant library (tools/build_variant.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributional_rl_decision_and_control_amd import learn_ops  # noqa: E402

dev = "cuda"
sup = torch.linspace(-1.0, 1.0, 51, device=dev)
tag = os.path.basename(os.environ.get("ASVRL_LIB", "default"))
for B in (64, 8192, 65536):
    pa = torch.softmax(torch.randn(B, 51, device=dev), 1)
    R = torch.randn(B, device=dev)
    nt = (torch.rand(B, device=dev) > 0.1).float()
    m = torch.empty_like(pa)
    for _ in range(5):
        learn_ops.c51_project(pa, R, nt, sup, out=m)
    n = 50   # captured in one graph: the host's per-call cost (~14 us through ctypes) stays out of the timing
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            learn_ops.c51_project(pa, R, nt, sup, out=m)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = 1e3 * e0.elapsed_time(e1) / n
    nbytes = B * (51 * 4 * 2 + 8)
    print(f"{tag} B={B}: {us:.2f} us/launch, {nbytes / us / 1e3:.0f} GB/s, {nbytes / us / 1e3 / 8000:.3f} of HBM",
          flush=True)
print("ok")
