#!/usr/bin/env python3
"""Root-cause probe for the hipGraphLaunch segfault of round 2.

Hypothesis: `torch.cuda.Stream()` hands out streams from a per-device pool of 32 (round-robin), so in a
long process (the full GPU suite) the "independent" streams of the captured schedule -- the capture
stream torch.cuda.graph creates once per process, VecTrainer's rollout stream, the learner's
SideStreams -- become the SAME hipStream once enough streams have been created. A captured fork/join
between two aliases of one stream is then a self-wait inside the capture.

Part 1 prints the pool's period. Part 2 runs the chained AC-IQN graph (unroll 2, 256 envs) in a child
process per case, with one alias forced (the rollout stream = the capture stream, a side stream = the
capture stream, a side stream = the rollout stream) and with the package's dedicated streams, and
compares each run's weights / losses with the joined schedule computed on unaliased streams.
Part 3 ("natural") builds trainers back to back in ONE process, as the suite does, with the torch pool.
Each child under its own timeout; the first crash ends the probe (no GPU step after a fault)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import faulthandler, sys, torch
faulthandler.enable()
sys.path.insert(0, ROOT)
from distributional_rl_decision_and_control_amd import streams as S
from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer

from distributional_rl_decision_and_control_amd.fused_update import ac_iqn_update_fused2, target_q


class PipeChain(VecTrainer):
    # round 2's reverted pipelined + chained schedule (parent of commit 3e2644b), restated for the probe
    # only: learn(k) consumes the batch produced beside learn(k-1)'s actor step on side stream 2,
    # sampled against the snapshot behind push(k) (waited for on that side stream)

    def _chained(self):
        return self.chain and self.overlap and self._fused_learner() and self.unroll % 2 == 0

    def learn(self, state=None, guard=0, actor_wait=None):
        if self.pipeline and not self._chained():
            return self._learn_pipelined(state, guard, actor_wait)
        saved, self.pipeline = self.pipeline, False
        try:
            return VecTrainer.learn(self, state, guard, actor_wait)
        finally:
            self.pipeline = saved

    def _produce2(self, nxt, state, guard, counter, counter_dev):
        st = self.fused2
        rows = self.replay.sample(self.B, seed=self.seed + 777, counter=counter, counter_dev=counter_dev,
                                  out=self.rows_buf[nxt], state=state, guard=guard, taus=self.taus_buf[nxt])
        target_q(st, rows, self.taus_buf[nxt][0], st.q_next_buf[nxt], st.na_p)

    def _chain_body(self):
        main = torch.cuda.current_stream(self.device)
        if self._streams is None:
            self._streams = (self.roll_stream(),) + self._roll_events()
        s_roll = self._streams[0]
        U = self.unroll
        ev_act = [torch.cuda.Event() for _ in range(U)]
        ev_snap = [torch.cuda.Event() for _ in range(U)]
        ev_learn = [torch.cuda.Event() for _ in range(U)]
        self._chain_events = (ev_act, ev_snap, ev_learn)
        s_roll.wait_stream(main)
        out = None
        for k in range(U):
            with torch.cuda.stream(s_roll):
                if k > 0:
                    s_roll.wait_event(ev_learn[k - 1])
                self.act()
                ev_act[k].record(s_roll)
                self.env.step(self.actions)
                self._push()
                self.ring_snap2[k % 2].copy_(self.replay.state)
                ev_snap[k].record(s_roll)
                self.env.auto_reset()
                self.env.advance_device()
            cur, nxt = k % 2, 1 - k % 2
            st = self.fused2
            self.counter_snap.copy_(self.learn_counter)

            def produce(k=k, nxt=nxt, snap_ready=ev_snap[k]):
                torch.cuda.current_stream(self.device).wait_event(snap_ready)
                self._produce2(nxt, self.ring_snap2[k % 2], self.E * self.R, 1, self.counter_snap)

            out = ac_iqn_update_fused2(st, self.local, self.actor_opt, self.critic_opt, self.critic_grads,
                                       self.actor_grads, self.rows_buf[cur], gamma=self.gamma, sync=self.sync,
                                       actor_wait=ev_act[k], taus=self.taus_buf[cur], q_next=st.q_next_buf[cur],
                                       produce=produce, counter=self.learn_counter)
            ev_learn[k].record(main)
        main.wait_stream(s_roll)
        return out

    def _capture(self):
        self.counter_snap = torch.zeros_like(self.learn_counter)
        # the graph's first learn consumes a batch produced right before the capture
        s = S.stream(self.device, "warmup")
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(3):
                self._iteration_body(True)
                self.env.advance_host()
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        self.ring_snap2[(self.unroll - 1) % 2].copy_(self.replay.state)
        self._produce2(0, self.ring_snap2[(self.unroll - 1) % 2], self.E * self.R, 0, self.learn_counter)
        with torch.cuda.graph(g, stream=S.capture_stream(self.device), capture_error_mode="thread_local"):
            self._graph_out = self._chain_body()
        self._graph = g


def run(chain, alias=None, pool=False, pipe=False):
    S.USE_TORCH_POOL = pool
    cls = PipeChain if pipe else VecTrainer
    tr = cls(n_envs=256, agent_type="AC-IQN", batch_size=256, num_tau=32, seed=21, graphs=True,
             unroll=2, chain=chain, buffer_size=256 * 5 * 40, learning_starts=512, pipeline=pipe)
    cap = S.capture_stream(tr.device)
    tr._streams = (cap if alias == "roll=capture" else tr.roll_stream(),) + tuple(tr._roll_events())
    if alias and alias.startswith("side"):
        i, other = int(alias[4]), alias.split("=")[1]
        tr.fused2.side.streams[i] = cap if other == "capture" else tr._streams[0]
    while tr.replay_size_host() < tr.learning_starts:
        tr.iteration()
    for _ in range(8):
        out = tr.iteration()
    torch.cuda.synchronize()
    p = torch.cat([q.detach().reshape(-1).float() for n in (tr.local.actor, tr.local.critic) for q in n.parameters()])
    return p, torch.stack([x.float().reshape(()) for x in out[:2]])

ref_p, ref_l = run(False)
if CASE.startswith("natural"):   # trainers back to back in one process, as in the suite
    pool, pipe = "dedicated" not in CASE, "pipe" in CASE
    for t in range(12):
        p, l = run(True, pool=pool, pipe=pipe)
        print("natural trainer", t, "equal" if torch.equal(p, ref_p) and torch.equal(l, ref_l) else "DIFFERENT",
              flush=True)
else:
    pipe = CASE.startswith("pipe")
    c = CASE.split(":")[-1]
    p, l = run(True, None if c in ("none", "dedicated") else c, pool=c != "dedicated", pipe=pipe)
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
    r = subprocess.run([sys.executable, "-c", POOL], capture_output=True, text=True, timeout=120)
    print("pool:", r.stdout.strip(), r.stderr.strip()[-300:] if r.returncode else "")
    cases = sys.argv[1:] or ["none", "dedicated", "roll=capture", "pipe:none", "pipe:roll=capture",
                             "pipe:side2=capture", "pipe:side2=roll", "natural", "natural-pipe",
                             "natural-pipe-dedicated"]
    for case in cases:
        code = f"ROOT = {ROOT!r}\nCASE = {case!r}\n" + CHILD
        print(f"=== {case}", flush=True)
        try:   # the child writes straight to our stdout / stderr (progress lines while it runs)
            r = subprocess.run([sys.executable, "-c", code], timeout=300)
        except subprocess.TimeoutExpired:
            print(f"{case:16s} TIMEOUT -- stopping", flush=True)
            return 1
        print(f"=== {case} rc={r.returncode}", flush=True)
        if r.returncode not in (0, 1):
            print("child crashed -- stopping", flush=True)
            return 2
    return 0


if __name__ == "__main__":
    sys.exit(main())
