"""Timeline of a rocprofv3 --kernel-trace CSV (one process, graph replays): per step, which
kernels run on which queue, the longest gaps, and each kernel symbol's total time -- used to read
the critical path of the pipelined schedule.
    python tools/trace_path.py gpurun_out/.../run_kernel_trace.csv [--last N]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n[-90:]


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")),
                   short(r["Kernel_Name"])))
    ks.sort()
    # the last N microseconds of the trace: steady-state replays
    last = float(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 20000.0
    t_end = max(k[1] for k in ks)
    win = [k for k in ks if k[0] >= t_end - last * 1000]
    t0 = win[0][0]
    by_q = defaultdict(list)
    for k in win:
        by_q[k[2]].append(k)
    for q, lst in by_q.items():
        busy = sum(b - a for a, b, _, _ in lst)
        print(f"queue {q}: {len(lst)} kernels, busy {busy / 1e3:.1f} us of {(lst[-1][1] - lst[0][0]) / 1e3:.1f} us")
    tot = defaultdict(float)
    for a, b, q, n in win:
        tot[(q, n)] += (b - a) / 1e3
    for (q, n), t in sorted(tot.items(), key=lambda x: -x[1])[:40]:
        print(f"  q{q} {t:10.1f} us  {n}")
    if "--dump" in sys.argv:
        for a, b, q, n in win[:400]:
            print(f"{(a - t0) / 1e3:9.1f} {(b - a) / 1e3:8.1f} q{q} {n}")


if __name__ == "__main__":
    main()
