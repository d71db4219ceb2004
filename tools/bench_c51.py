#!/usr/bin/env python3
"""C51 projection kernel alone (asvrl_c51_project) at B in {64, 8192, 65536}: 50 eager launches per
size, for rocprofv3 --kernel-trace --stats (the kernel durations are the measurement)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributional_rl_decision_and_control_amd import learn_ops  # noqa: E402

dev = "cuda"
sup = torch.linspace(-1.0, 1.0, 51, device=dev)
for B in (64, 8192, 65536):
    pa = torch.softmax(torch.randn(B, 51, device=dev), 1)
    R = torch.randn(B, device=dev)
    nt = (torch.rand(B, device=dev) > 0.1).float()
    m = torch.empty_like(pa)
    for _ in range(50):
        learn_ops.c51_project(pa, R, nt, sup, out=m)
    torch.cuda.synchronize()
print("ok")
