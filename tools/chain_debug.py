#!/usr/bin/env python3
"""Which (envs, batch, unroll) make the chained AC-IQN schedule differ from the joined one (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_chain_schedule_gpu import _run  # noqa: E402

for E, B, U, it in [(256, 256, 2, 8), (256, 256, 4, 8), (256, 256, 10, 20), (4096, 4096, 2, 8), (4096, 4096, 10, 20)]:
    a, pa, la = _run("AC-IQN", True, it, n_envs=E, batch=B, unroll=U)
    del a
    b, pb, lb = _run("AC-IQN", False, it, n_envs=E, batch=B, unroll=U)
    del b
    print(f"E={E} B={B} U={U} it={it}: losses equal {torch.equal(la, lb)} {la.tolist()} {lb.tolist()} "
          f"params max diff {float((pa - pb).abs().max()):.3e}", flush=True)
