# Backs DESIGN §8 "Launch gaps": a sort replayed as a HIP graph is no faster than direct launches.
"""dev/graph_lab.py -- launch-gap cost: the same device sort timed as direct launches and as a
replayed HIP graph (torch.cuda.CUDAGraph capture of rsort_sort_planned), C2 and C3 shapes."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cuda.radixsort_amd"))
import torch
import radixsort as rs

def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps

for n, k in ((1 << 26, 4), (1 << 30, 8), (1 << 24, 8)):
    x = torch.empty(n, dtype=torch.int32, device="cuda")
    rs.gen_uniform(x, 0x5EED)
    y = torch.empty_like(x)
    p = rs.plan(n, k)
    ws = rs.workspace(p.workspace_bytes)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(3):
            rs.sort_device(x, y, k, ws=ws, plan_=p)
        torch.cuda.synchronize()
        direct = timeit(lambda: rs.sort_device(x, y, k, ws=ws, plan_=p), 20)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            rs.sort_device(x, y, k, ws=ws, plan_=p)
        g.replay()
        torch.cuda.synchronize()
        ok = bool(torch.all(y[1:].to(torch.int64) & 0xFFFFFFFF >= y[:-1].to(torch.int64) & 0xFFFFFFFF))
        graph = timeit(g.replay, 20)
    print(f"n=2^{n.bit_length()-1} k={k}: direct {direct:.4f} ms, graph {graph:.4f} ms, sorted={ok}", flush=True)
