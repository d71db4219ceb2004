"""Where the driver's short timed region loses time: the bench's AC-IQN step (4096 envs, B = 4096, chained
graph of U iterations), timed from a synchronised start as bench.py does, with the host's submission time of
each graph replay and HIP events on the capture's origin stream.

    python tools/launch_probe.py [--unroll 10] [--replays 2] [--trials 8]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--unroll", type=int, default=10)
    ap.add_argument("--replays", type=int, default=2)
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--warm-replays", type=int, default=2)
    ap.add_argument("--sequence", action="store_true", help="print every trial in order (no idle variants)")
    ap.add_argument("--pre", default="none", choices=["none", "upload", "burn"],
                    help="before the trials: hipGraphUpload of the captured graph, or ~100 ms of unrelated GPU work")
    a = ap.parse_args()
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    dev = torch.device("cuda", 0)
    tr = VecTrainer(n_envs=4096, agent_type="AC-IQN", num_robots=5, num_obs=4, width=55.0, batch_size=4096,
                    num_tau=32, seed=1000, device=dev, graphs=True, learning_starts=4096, unroll=a.unroll)
    while tr.replay_size_host() < tr.learning_starts:
        tr.iteration()
    for _ in range(a.warm_replays * a.unroll):
        tr.iteration()
    torch.cuda.synchronize(dev)
    g = tr._graph
    stream = torch.cuda.current_stream(dev)
    if a.pre == "upload":
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
        torch.cuda.synchronize(dev)
        print("hipGraphUpload rc", rc, flush=True)
    elif a.pre == "burn":
        x = torch.randn(4096, 4096, device=dev)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.1:
            for _ in range(10):
                x = torch.tanh(x @ x * 1e-3)
            torch.cuda.synchronize(dev)
        del x
    for idle_ms in ((0.0,) if a.sequence else (0.0, 5.0)):
        walls, hosts, evs = [], [], []
        for _ in range(a.trials):
            torch.cuda.synchronize(dev)
            if idle_ms:
                time.sleep(idle_ms * 1e-3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            hs = []
            for _ in range(a.replays):
                h0 = time.perf_counter()
                g.replay()
                hs.append(time.perf_counter() - h0)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            walls.append(time.perf_counter() - t0)
            hosts.append(hs)
            evs.append(e0.elapsed_time(e1) * 1e-3)
        n = a.replays * a.unroll
        if a.sequence:
            print("trial ms/step in order:", [round(1e3 * w / n, 4) for w in walls], flush=True)
        med = sorted(walls)[len(walls) // 2]
        print(f"idle {idle_ms} ms: unroll {a.unroll} x {a.replays} replays: wall {1e3 * med / n:.4f} ms/step "
              f"(min {1e3 * min(walls) / n:.4f}), events {1e3 * sorted(evs)[len(evs) // 2] / n:.4f} ms/step, "
              f"host submit per replay (us) first {1e6 * sorted(h[0] for h in hosts)[len(hosts) // 2]:.0f} "
              f"rest {[round(1e6 * x) for x in hosts[-1][1:]]}", flush=True)


if __name__ == "__main__":
    main()
