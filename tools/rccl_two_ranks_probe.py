"""Probe: can two RCCL ranks share one GPU (the only layout a 1-GPU box offers)? Each rank all-reduces
(AVG) a small device tensor on cuda:0 and prints the result; the parent reports each rank's exit code.
    python tools/rccl_two_ranks_probe.py"""
import os
import socket
import subprocess
import sys


def worker(rank, port):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=2, device_id=dev)
    x = torch.full((1024,), float(rank + 1), device=dev)
    dist.all_reduce(x, op=dist.ReduceOp.AVG)
    torch.cuda.synchronize()
    print(f"rank {rank}: avg {x[0].item()} (want 1.5)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        worker(int(sys.argv[1]), sys.argv[2])
        sys.exit(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = [subprocess.Popen([sys.executable, __file__, str(r), port]) for r in range(2)]
    codes = [p.wait(timeout=120) for p in procs]
    print("exit codes", codes, flush=True)
    sys.exit(0 if all(c == 0 for c in codes) else 1)
