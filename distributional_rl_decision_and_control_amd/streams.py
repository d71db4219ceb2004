"""Dedicated HIP streams for the captured rollout + learn schedule.

`torch.cuda.Stream()` does not create a stream: it hands out the next of a per-device pool of 32
(round-robin). In one long process -- the full GPU test suite, a training script that builds several
trainers -- the streams the captured schedule treats as independent (the capture stream
torch.cuda.graph creates once per process, VecTrainer's rollout stream, the learner's side streams)
therefore become the SAME hipStream once ~32 streams have been handed out, and a fork/join between two
aliases of one stream turns into a self-wait inside the capture (round 2's hipGraphLaunch segfault,
DESIGN.md section 6; `tools/graph_stream_probe.py` forces each alias).

Here every role gets its own stream, created once per (device, role) with hipStreamCreateWithFlags
(non-blocking, like torch's pool streams) and wrapped as a torch.cuda.ExternalStream: no other code in
the process can be handed the same stream. The streams live for the process.
"""
import ctypes as C
import os

import torch

# the probe (tools/graph_stream_probe.py) switches to torch's pool to show the aliasing
USE_TORCH_POOL = False
# per-role HIP stream priority ("role=high|low,...", e.g. "capture=high,roll=low"; unset: every stream at
# the default priority), read when a role's stream is first created
PRIORITIES = os.environ.get("ASVRL_STREAM_PRIORITY", "")

_HIP = None
_STREAMS = {}
_NON_BLOCKING = 1   # hipStreamNonBlocking


def _hip():
    global _HIP
    if _HIP is None:
        torch.cuda.init()   # the HIP runtime torch loaded (one runtime per process: same soname)
        _HIP = C.CDLL("libamdhip64.so.7")
        _HIP.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
        _HIP.hipStreamCreateWithFlags.restype = C.c_int
        _HIP.hipStreamCreateWithPriority.argtypes = [C.POINTER(C.c_void_p), C.c_uint, C.c_int]
        _HIP.hipStreamCreateWithPriority.restype = C.c_int
        _HIP.hipDeviceGetStreamPriorityRange.argtypes = [C.POINTER(C.c_int), C.POINTER(C.c_int)]
        _HIP.hipDeviceGetStreamPriorityRange.restype = C.c_int
    return _HIP


def _priority(role):
    """The numeric HIP priority of `role` from PRIORITIES, or None (lower numbers run first)."""
    for item in PRIORITIES.split(","):
        name, _, level = item.partition("=")
        if name.strip() == str(role) and level.strip() in ("high", "low"):
            least, greatest = C.c_int(), C.c_int()
            if _hip().hipDeviceGetStreamPriorityRange(C.byref(least), C.byref(greatest)) != 0:
                raise RuntimeError("hipDeviceGetStreamPriorityRange failed")
            return greatest.value if level.strip() == "high" else least.value
    return None


def stream(device, role):
    """The process-wide stream of `role` (a hashable name) on `device`."""
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if USE_TORCH_POOL:
        return torch.cuda.Stream(device=dev)
    key = (dev.index, role)
    s = _STREAMS.get(key)
    if s is None:
        h = C.c_void_p()
        prio = _priority(role)
        with torch.cuda.device(dev):
            if prio is None:
                rc = _hip().hipStreamCreateWithFlags(C.byref(h), _NON_BLOCKING)
            else:
                rc = _hip().hipStreamCreateWithPriority(C.byref(h), _NON_BLOCKING, prio)
        if rc != 0:
            raise RuntimeError(f"hipStreamCreate failed ({rc})")
        s = torch.cuda.ExternalStream(h.value, device=dev)
        _STREAMS[key] = s
    return s


def capture_stream(device):
    """The stream every VecTrainer graph is captured on (instead of torch.cuda.graph's pool stream)."""
    if USE_TORCH_POOL:   # what torch.cuda.graph uses when no stream is given
        g = torch.cuda.graphs.graph
        if g.default_capture_stream is None:
            g.default_capture_stream = torch.cuda.Stream()
        return g.default_capture_stream
    return stream(device, "capture")
