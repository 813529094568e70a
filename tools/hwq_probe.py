"""Which HIP streams share a hardware queue (and so serialize), and what a captured two-branch graph does:
two one-wave spin kernels (torch.cuda._sleep) on streams a and b take 1x a spin when a and b sit on
different hardware queues and 2x when they share one.  Streams: torch's pool (normal / high priority),
hipExtStreamCreateWithCUMask with every CU set, and the caller's default stream; then a forked
two-branch hipGraph captured several times, and one graph per branch replayed on its own stream.
  python tools/hwq_probe.py"""
import ctypes
import os
import time

import torch

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(dev).multi_processor_count
print("GPU_MAX_HW_QUEUES =", os.environ.get("GPU_MAX_HW_QUEUES"), " CUs", NCU, flush=True)


def cumask_stream():
    s = ctypes.c_void_p()
    n = (NCU + 31) // 32
    mask = (ctypes.c_uint32 * n)(*([0xFFFFFFFF] * n))
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(n), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


# calibrate: one spin of about 2 ms
C = 1 << 20
torch.cuda._sleep(C)
torch.cuda.synchronize()
t0 = time.perf_counter()
torch.cuda._sleep(C)
torch.cuda.synchronize()
one = time.perf_counter() - t0
C = int(C * 2e-3 / one)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    torch.cuda._sleep(C)
torch.cuda.synchronize()
one = (time.perf_counter() - t0) / 3
print(f"spin {one * 1e3:.2f} ms", flush=True)


def pair(a, b):
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(a):
            torch.cuda._sleep(C)
        with torch.cuda.stream(b):
            torch.cuda._sleep(C)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best / one


def matrix(name, sts):
    print(f"## {name}: pair time / one spin (1 = concurrent, 2 = same queue); row/col 0 = default stream",
          flush=True)
    allst = [torch.cuda.default_stream(dev)] + sts
    for i in range(len(allst)):
        print("  " + " ".join(f"{pair(allst[i], allst[j]):4.1f}" if j > i else "   -" for j in range(len(allst))),
              flush=True)


matrix("torch pool, priority 0", [torch.cuda.Stream(device=dev) for _ in range(6)])
matrix("torch pool, priority -1", [torch.cuda.Stream(device=dev, priority=-1) for _ in range(6)])
matrix("hipExtStreamCreateWithCUMask (all CUs)", [cumask_stream() for _ in range(4)])


def time_replay(fn):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best / one


print("## one graph, two forked branches (torch pool streams a, b), captured 6 times", flush=True)
res = []
for _ in range(6):
    a, b = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream(dev)
        for st in (a, b):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                torch.cuda._sleep(C)
        for st in (a, b):
            cur.wait_stream(st)
    res.append(time_replay(g.replay))
print("  " + " ".join(f"{r:.2f}" for r in res), flush=True)


def per_branch(mk, name):
    res = []
    for _ in range(4):
        sts = [mk(), mk()]
        gs = []
        for st in sts:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                torch.cuda._sleep(C)
            gs.append(g)

        def run():
            cur = torch.cuda.current_stream(dev)
            for st, g in zip(sts, gs):
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    g.replay()
            for st in sts:
                cur.wait_stream(st)
        res.append(time_replay(run))
    print(f"## one graph per branch, replayed on its own stream ({name}): " + " ".join(f"{r:.2f}" for r in res),
          flush=True)


per_branch(lambda: torch.cuda.Stream(device=dev), "torch pool")
per_branch(cumask_stream, "CU-mask streams")

print("## pool offset k: part streams = the next two pool streams; eager pair, then a forked graph captured on a"
      " fresh side stream (the GraphReplay pattern) replayed on the default stream", flush=True)
for k in range(10):
    for _ in range(k):
        torch.cuda.Stream(device=dev)
    a, b = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)
    eager = pair(a, b)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            cur = torch.cuda.current_stream(dev)
            for st in (a, b):
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    torch.cuda._sleep(C)
            for st in (a, b):
                cur.wait_stream(st)
    print(f"  k={k}: eager {eager:.2f}  graph {time_replay(g.replay):.2f}", flush=True)
