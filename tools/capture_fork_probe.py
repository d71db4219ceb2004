#!/usr/bin/env python3
"""Probe which SideStreams fork/join patterns HIP graph capture accepts (each in its own process)."""
import subprocess
import sys

CASES = {
    "A_one_fork_join": "with sd.on(0): k()\nsd.join(0)",
    "B_refork_after_join": "with sd.on(0): k()\nsd.join(0)\nk()\nwith sd.on(0): k()\nsd.join(0)",
    "C_two_forks_joined": "with sd.on(0): k()\nwith sd.on(1): k()\nk()\nsd.join(0)\nsd.join(1)",
    "D_refork_unjoined": "with sd.on(1): k()\nk()\nwith sd.on(1): k()\nsd.join(1)",
    "E_update_shape": ("with sd.on(0): k()\nwith sd.on(1): k()\nk()\nsd.join(0)\nk()\nwith sd.on(0): k()\nk()\n"
                       "with sd.on(1): k()\nsd.join()"),
    "F_inside_learn_stream": "LEARN",
    "G_learn_and_rollout": "LEARN2",
    "H_learn_A_only": "LEARN_A",
}

BODY = r"""
import sys, torch
sys.path.insert(0, '.')
from distributional_rl_decision_and_control_amd.fused_update import SideStreams
x = torch.zeros(1 << 20, device='cuda')
sd = SideStreams('cuda', 2)
def k():
    x.add_(1.0)
learn, roll = torch.cuda.Stream(), torch.cuda.Stream()
y = torch.zeros(1 << 20, device='cuda')
def body():
    if CASE.startswith('LEARN'):
        main = torch.cuda.current_stream()
        learn.wait_stream(main)
        roll.wait_stream(main)
        if CASE == 'LEARN2':
            with torch.cuda.stream(roll):
                y.add_(2.0)
        with torch.cuda.stream(learn):
            exec(CASES_E if CASE != 'LEARN_A' else "with sd.on(0): k()\nsd.join(0)")
        main.wait_stream(learn)
        main.wait_stream(roll)
    else:
        exec(CASE)
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
g.replay(); torch.cuda.synchronize(); print('ok', float(x[0]))
"""

for name, case in CASES.items():
    code = f"CASE = {case!r}\nCASES_E = {CASES['E_update_shape']!r}\n" + BODY
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    err = [ln for ln in r.stderr.splitlines() if "amdgpu.ids" not in ln][-3:] if r.returncode else ""
    print(f"{name:24s} rc={r.returncode} {r.stdout.strip()[-40:]} {err}")
