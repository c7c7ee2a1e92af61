"""How fast does a captured graph feed its kernels to the GPU?  (GPU box, no profiler)
    python tools/probe/graph_rate.py
Graphs of N back-to-back one-block kernels (torch.cuda._sleep of ~1 us, ~20 us) in one chain, and
in two branches of N/2, timed with events around replay; the same N launched eagerly on a stream.
If the per-node time stays ~15 us for the 1 us kernels, the graph's submission rate -- not the
kernels -- sets the length of a step of many short kernels."""
import torch

dev = torch.device("cuda:0")
torch.cuda.init()
side, cap = torch.cuda.Stream(), torch.cuda.Stream()


def build(n, cycles, branches):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        g.capture_begin()
        cur = torch.cuda.current_stream()
        if branches == 2:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                for _ in range(n // 2):
                    torch.cuda._sleep(cycles)
            for _ in range(n - n // 2):
                torch.cuda._sleep(cycles)
            cur.wait_stream(side)
        else:
            for _ in range(n):
                torch.cuda._sleep(cycles)
        g.capture_end()
    return g


def timed(fn, reps=20):
    s = cap
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for cycles in (100, 40_000):
    one = timed(lambda: torch.cuda._sleep(cycles), reps=200)
    print(f"sleep({cycles}): one eager launch {one:.1f} us", flush=True)
    for n in (50, 200):
        eager = timed(lambda: [torch.cuda._sleep(cycles) for _ in range(n)], reps=10)
        g1 = build(n, cycles, 1)
        g2 = build(n, cycles, 2)
        t1 = timed(g1.replay)
        t2 = timed(g2.replay)
        print(f"  N={n}: eager {eager:8.1f} us ({eager / n:5.1f}/node)  graph chain {t1:8.1f} us ({t1 / n:5.1f}/node)"
              f"  graph 2 branches {t2:8.1f} us ({t2 / n:5.1f}/node)", flush=True)
