#!/usr/bin/env python3
"""Root-cause probe for round 2's captured-graph segfault.

Cause: `torch.cuda.Stream()` hands out streams from a per-device pool of 32 (round-robin), so in one
long process (the full GPU suite) two streams a captured schedule treats as independent can be the
SAME hipStream. Round 2's pipelined + chained learner forked a side stream from the capture stream and
made it wait on an event of the rollout stream; when the side stream and the rollout stream were one
stream, ROCm's capture crashed (profiles/r03_graph_stream_probe.log: the trainer-level case
"pipe:side2=roll" segfaulted in capture_end; every unaliased case and the dedicated streams were
bit-identical to the joined schedule; that run used this file at commit 125d91f, whose PipeChain class
restated the reverted schedule).

This file keeps a minimal, trainer-free form of the pattern and the trainer-level check of the current
schedule:
  pool            the pool's period (torch.cuda.Stream() #32 is #0 again)
  mini:<case>     main -> fork R (rollout) -> record ev; fork S from main, S waits ev, S joins main;
                  with S a distinct stream, S == R (pool alias), S == the capture stream, or the
                  package's dedicated streams (streams.py); checks the replayed result
  trainer:<case>  the chained AC-IQN graph (unroll 2, 256 envs) vs the joined schedule, with the
                  rollout stream aliased to the capture stream, and on the dedicated streams
Each case runs in its own child process under a timeout; the first crash ends the probe."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MINI = r"""
import faulthandler, sys, torch
faulthandler.enable()
sys.path.insert(0, ROOT)
from distributional_rl_decision_and_control_amd import streams as S
x = torch.zeros(1 << 16, device="cuda")
if CASE == "dedicated":
    C, R, SS = S.capture_stream("cuda"), S.stream("cuda", "roll"), S.stream("cuda", "side")
else:
    C, R = torch.cuda.Stream(), torch.cuda.Stream()
    SS = {"distinct": torch.cuda.Stream(), "side=roll": R, "side=capture": C}[CASE]
ev = torch.cuda.Event()
def body():
    main = torch.cuda.current_stream()
    R.wait_stream(main)
    with torch.cuda.stream(R):
        x.add_(1.0)
        ev.record(R)
    SS.wait_stream(main)
    with torch.cuda.stream(SS):
        torch.cuda.current_stream().wait_event(ev)
        x.mul_(2.0)
    main.wait_stream(SS)
    main.wait_stream(R)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=C):
    body()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print(CASE, "x =", float(x[0]), "(expected 14.0)", flush=True)
"""

TRAINER = r"""
import faulthandler, sys, torch
faulthandler.enable()
sys.path.insert(0, ROOT)
from distributional_rl_decision_and_control_amd import streams as S
from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer

def run(chain, alias=None, pool=False):
    S.USE_TORCH_POOL = pool
    tr = VecTrainer(n_envs=256, agent_type="AC-IQN", batch_size=256, num_tau=32, seed=21, graphs=True,
                    unroll=2, chain=chain, buffer_size=256 * 5 * 40, learning_starts=512)
    cap = S.capture_stream(tr.device)
    tr._streams = (cap if alias == "roll=capture" else tr.roll_stream(),) + tuple(tr._roll_events())
    while tr.replay_size_host() < tr.learning_starts:
        tr.iteration()
    for _ in range(8):
        out = tr.iteration()
    torch.cuda.synchronize()
    p = torch.cat([q.detach().reshape(-1).float() for n in (tr.local.actor, tr.local.critic) for q in n.parameters()])
    return p, torch.stack([x.float().reshape(()) for x in out[:2]])

ref_p, ref_l = run(False)
p, l = run(True, None if CASE == "dedicated" else CASE, pool=CASE != "dedicated")
print(CASE, "equal" if torch.equal(p, ref_p) and torch.equal(l, ref_l) else
      "DIFFERENT max|dp|=%g" % float((p - ref_p).abs().max()), flush=True)
"""

POOL = r"""
import torch
torch.cuda.init()
hs = [torch.cuda.Stream().cuda_stream for _ in range(70)]
first = {}
for i, h in enumerate(hs):
    if h in first:
        print("torch.cuda.Stream() #%d is the same hipStream as #%d (period %d)" % (i, first[h], i - first[h]))
        break
    first[h] = i
else:
    print("no repeat in 70 streams")
"""


def main():
    cases = sys.argv[1:] or ["pool", "mini:distinct", "mini:dedicated", "mini:side=capture", "trainer:roll=capture",
                             "trainer:dedicated", "mini:side=roll"]
    for case in cases:
        kind, _, sub = case.partition(":")
        src = {"pool": POOL, "mini": MINI, "trainer": TRAINER}[kind]
        code = f"ROOT = {ROOT!r}\nCASE = {sub!r}\n" + src
        print(f"=== {case}", flush=True)
        try:   # the child writes straight to our stdout / stderr
            r = subprocess.run([sys.executable, "-c", code], timeout=300)
        except subprocess.TimeoutExpired:
            print(f"{case} TIMEOUT -- stopping", flush=True)
            return 1
        print(f"=== {case} rc={r.returncode}", flush=True)
        if r.returncode not in (0, 1):
            print("child crashed -- stopping", flush=True)
            return 2
    return 0


if __name__ == "__main__":
    sys.exit(main())
