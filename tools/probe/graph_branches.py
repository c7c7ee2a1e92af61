"""Do the two branches of a captured two-stream graph run concurrently? (GPU box)
    python tools/probe/graph_branches.py
Branch A: NA sleep kernels of TA cycles (one block each) on a side stream; branch B: NB of TB on
the capturing stream.  Prints the replay time of: one graph with both branches (A captured first
/ B first), each branch alone, and two single-branch graphs replayed on two streams."""
import time

import torch

dev = torch.device("cuda:0")
NA, TA, NB, TB = 40, 200_000, 120, 60_000


def chain(n, cyc):
    for _ in range(n):
        torch.cuda._sleep(cyc)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def two_branch(a_first):
    side = torch.cuda.Stream()
    cap = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        g.capture_begin()
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        if a_first:
            with torch.cuda.stream(side):
                chain(NA, TA)
            chain(NB, TB)
        else:
            chain(NB, TB)
            with torch.cuda.stream(side):
                chain(NA, TA)
        cur.wait_stream(side)
        g.capture_end()
    return g


def single(n, cyc):
    cap = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        g.capture_begin()
        chain(n, cyc)
        g.capture_end()
    return g


ga, gb = single(NA, TA), single(NB, TB)
print(f"A alone {timed(ga.replay):.2f} ms, B alone {timed(gb.replay):.2f} ms", flush=True)
for af in (True, False):
    g = two_branch(af)
    print(f"one graph, {'A' if af else 'B'} captured first: {timed(g.replay):.2f} ms", flush=True)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def two_graphs():
    main = torch.cuda.current_stream()
    s1.wait_stream(main)
    s2.wait_stream(main)
    with torch.cuda.stream(s1):
        ga.replay()
    with torch.cuda.stream(s2):
        gb.replay()
    main.wait_stream(s1)
    main.wait_stream(s2)


print(f"two graphs on two streams: {timed(two_graphs):.2f} ms", flush=True)


def eager():
    main = torch.cuda.current_stream()
    s1.wait_stream(main)
    with torch.cuda.stream(s1):
        chain(NA, TA)
    chain(NB, TB)
    main.wait_stream(s1)


print(f"eager two streams: {timed(eager):.2f} ms", flush=True)
