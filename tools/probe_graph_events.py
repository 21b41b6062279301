#!/usr/bin/env python
"""Which cross-stream signalling out of a replayed HIP graph works on this
stack (diagnostic for the graph step's comm_mode "event", engine/graphs.py)?

    python tools/probe_graph_events.py <case>

Cases (each meant to run in its own process under a time limit):
  external   torch.cuda.Event(external=True) recorded inside the capture
  keepgraph  CUDAGraph(keep_graph=True): capture_end without instantiation,
             raw graph handle available (nodes could be added before instantiate)
  waitvalue  hipStreamWaitValue32 on a second stream against a flag a kernel
             writes inside the replay (stream memory operations)
Prints one line "<case> ok|FAIL <detail>".
"""
import ctypes
import sys

import torch


def external():
    dev = torch.device("cuda", 0)
    a = torch.zeros(64 << 20, device=dev)
    cnt = torch.zeros(1, device=dev)
    seen = torch.zeros(1, device=dev)
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    from distributed_3d_diffusion_pytorch_amd.ops.hip_impl import ExternalEvent
    ev = ExternalEvent()
    g = torch.cuda.CUDAGraph()
    a.mul_(0.5).add_(1.0)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(16):
            a.mul_(0.5).add_(1.0)
        cnt.add_(1.0 + 0.0 * a[:1])
        ev.record()
        a.mul_(0.5).add_(1.0)
    s = torch.cuda.Stream()
    for rep in range(3):
        g.replay()
        ev.wait_on(s)
        with torch.cuda.stream(s):
            seen.copy_(cnt)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if seen.item() != rep + 1:
            return f"stale counter {seen.item()} at replay {rep}"
    return None


def keepgraph():
    g = torch.cuda.CUDAGraph(keep_graph=True)
    x = torch.zeros(16, device="cuda")
    x.add_(0.0)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        x.add_(1.0)
    h = g.raw_cuda_graph()
    g.instantiate()
    g.replay()
    torch.cuda.synchronize()
    if x[0].item() != 1.0:
        return f"replay result {x[0].item()}"
    print(f"raw graph handle {h:#x}")
    return None


def waitvalue():
    hip = ctypes.CDLL("libamdhip64.so")
    fn = hip.hipStreamWaitValue32
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
    fn.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    a = torch.zeros(64 << 20, device=dev)
    flag = torch.zeros(4, dtype=torch.int32, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    seen = torch.zeros(1, dtype=torch.int32, device=dev)
    g = torch.cuda.CUDAGraph()
    a.mul_(0.5).add_(1.0)
    flag[:1].copy_(step + (a[:1] * 0).int())
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(16):
            a.mul_(0.5).add_(1.0)
        flag[:1].copy_(step + (a[:1] * 0).int())
        a.mul_(0.5).add_(1.0)
    s = torch.cuda.Stream()
    for rep in range(1, 4):
        step.fill_(rep)
        g.replay()
        rc = fn(ctypes.c_void_p(s.cuda_stream), ctypes.c_void_p(flag.data_ptr()), rep, 1, 0xFFFFFFFF)  # 1: >=
        if rc != 0:
            return f"hipStreamWaitValue32 rc {rc}"
        with torch.cuda.stream(s):
            seen.copy_(flag[:1])
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if seen.item() != rep:
            return f"saw {seen.item()} at replay {rep}"
    return None


if __name__ == "__main__":
    case = sys.argv[1]
    try:
        err = {"external": external, "keepgraph": keepgraph, "waitvalue": waitvalue}[case]()
    except Exception as e:      # noqa: BLE001
        err = f"{type(e).__name__}: {str(e).splitlines()[0][:200]}"
    print(f"{case} {'ok' if err is None else 'FAIL ' + err}", flush=True)
