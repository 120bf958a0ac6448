"""Probe: the device gap between two back-to-back replays of HIP graphs, against the number of kernel nodes in
the graph.  Graphs of N small kernels (each ~20 us of work), replayed twice in a row on one stream with the host
far ahead; prints the gap between the first replay's end event and the second's start event.  Also: the same
for two DIFFERENT graphs (A then B), and for one graph of N kernels split in two graphs of N/2.
Usage: python scripts/graph_gap_probe.py"""
import torch

dev = torch.device("cuda:0")
x = torch.randn(1 << 20, device=dev)


def make_graph(n):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    y = x.clone()
    with torch.cuda.stream(s):
        for _ in range(3):  # warm
            y.mul_(1.0000001)
        torch.cuda.synchronize()
        g.capture_begin()
        for _ in range(n):
            y.mul_(1.0000001).add_(1e-7)
        g.capture_end()
    torch.cuda.synchronize()
    return g, y


def gaps(ga, gb, reps=6):
    cur = torch.cuda.current_stream()
    ev = []
    # a long kernel first so the host is far ahead of the device
    z = torch.randn(4096, 4096, device=dev)
    for _ in range(30):
        z = z @ z
        z = z / z.norm()
    for k in range(reps):
        g = ga if k % 2 == 0 else gb
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(cur)
        g.replay()
        e.record(cur)
        ev.append((s, e))
    torch.cuda.synchronize()
    run = [round(s.elapsed_time(e), 3) for s, e in ev]
    gap = [round(ev[k][1].elapsed_time(ev[k + 1][0]), 3) for k in range(len(ev) - 1)]
    return run, gap


import ctypes  # noqa: E402
_hip = ctypes.CDLL("libamdhip64.so")
_hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
_hip.hipGraphUpload.restype = ctypes.c_int


def fresh(k, n, upload):
    """k graphs of n kernels, each replayed once, captured just before (as bench.py does per step); upload: each
    graph uploaded on a side stream right after its capture."""
    cur = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    z = torch.randn(4096, 4096, device=dev)
    for _ in range(30):
        z = z @ z
        z = z / z.norm()
    ev, keep = [], []
    for i in range(k):
        g, y = make_graph_nosync(n)
        if upload:
            rc = _hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()), ctypes.c_void_p(side.cuda_stream))
            assert rc == 0, rc
            u = torch.cuda.Event()
            u.record(side)
            cur.wait_event(u)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(cur)
        g.replay()
        e.record(cur)
        ev.append((s, e))
        keep.append((g, y))
    torch.cuda.synchronize()
    run = [round(s.elapsed_time(e), 3) for s, e in ev]
    gap = [round(ev[j][1].elapsed_time(ev[j + 1][0]), 3) for j in range(len(ev) - 1)]
    return run, gap


_cap = torch.cuda.Stream()


def make_graph_nosync(n):
    g = torch.cuda.CUDAGraph()
    y = x.clone()
    with torch.cuda.stream(_cap):
        g.capture_begin()
        for _ in range(n):
            y.mul_(1.0000001).add_(1e-7)
        g.capture_end()
    return g, y


for n in (50, 450, 900, 1800):
    ga, _ = make_graph(n)
    gb, _ = make_graph(n)
    run, gap = gaps(ga, ga)
    print(f"N={n:5d} same graph     replay ms {run}  gap ms {gap}", flush=True)
    run, gap = gaps(ga, gb)
    print(f"N={n:5d} two graphs     replay ms {run}  gap ms {gap}", flush=True)
    for up in (False, True):
        run, gap = fresh(5, n, up)
        print(f"N={n:5d} fresh graphs, upload {int(up)}: replay ms {run}  gap ms {gap}", flush=True)
