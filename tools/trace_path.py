"""Per-step timeline of a rocprofv3 --kernel-trace CSV (one process, graph replays): where the
step's wall time goes on each queue, to read the critical path of the pipelined schedule.

    python tools/trace_path.py gpurun_out/.../kernel_trace.csv [--steps 2] [--dump]

A step ends at each clamp_adam launch (the optimizer, once per train step on the main queue).
Per step: wall time (adam end to adam end), per queue busy time and span, the main queue's idle
gaps (> 2 us, with the kernel that ends each), and the kernel symbols by total time."""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    """Readable kernel identifier: demangled `imgcap::foo<...>` -> foo<...> (args trimmed),
    mangled _ZN6imgcap..3fooI.. -> foo, torch kernels -> their functor."""
    n = name.strip()
    m = re.match(r"_ZN(?:\d+\w+?)*?6imgcap(?:12_GLOBAL__N_1)?(\d+)", n)
    if m:
        k = int(m.group(1))
        rest = n[m.end():]
        return rest[:k]
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*$", "", n)
    if "imgcap::" in n:
        n = n[n.index("imgcap::") + 8:]
        return n[:60]
    f = re.search(r"at::native::(?:\w+::)*(\w+Functor\w*|\w+_kernel\w*)", n)
    if f:
        return "torch:" + f.group(1)
    return n[:60]


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 2
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r.get("Queue_Id", r.get("Stream_Id", "?")), short(r["Kernel_Name"])) for r in rows)
    adams = [k for k in ks if k[3].startswith("clamp_adam")]
    if len(adams) < nsteps + 1:
        print("not enough steps in the trace")
        return
    for si in range(len(adams) - nsteps, len(adams)):
        t0, t1 = adams[si - 1][1], adams[si][1]
        win = [k for k in ks if k[0] >= t0 and k[0] < t1]
        print(f"=== step {si}: wall {(t1 - t0) / 1e3:.1f} us, {len(win)} kernels")
        by_q = defaultdict(list)
        for k in win:
            by_q[k[2]].append(k)
        for q, lst in sorted(by_q.items(), key=lambda x: -len(x[1])):
            busy = sum(b - a for a, b, _, _ in lst)
            print(f"  queue {q}: {len(lst)} kernels, busy {busy / 1e3:.1f} us, span "
                  f"{(lst[0][0] - t0) / 1e3:.1f} .. {(lst[-1][1] - t0) / 1e3:.1f} us")
        main_q = max(by_q, key=lambda q: len(by_q[q]))
        lst = by_q[main_q]
        gaps = []
        prev_end, prev_name = t0, "(step start)"
        for a, b, _, n in lst:
            if a - prev_end > 2000:
                gaps.append(((a - prev_end) / 1e3, prev_name, n, (prev_end - t0) / 1e3))
            prev_end, prev_name = max(prev_end, b), n
        print(f"  main queue {main_q} idle gaps > 2 us: " + "; ".join(
            f"{g:.1f} us at {at:.0f} after {p} before {n}" for g, p, n, at in gaps))
        tot = defaultdict(float)
        cnt = defaultdict(int)
        for a, b, q, n in win:
            tot[(q, n)] += (b - a) / 1e3
            cnt[(q, n)] += 1
        for (q, n), t in sorted(tot.items(), key=lambda x: -x[1])[:24]:
            print(f"    q{q} {t:9.1f} us  x{cnt[(q, n)]:<3d} {n}")
        if "--dump" in sys.argv:
            for a, b, q, n in win:
                print(f"    {(a - t0) / 1e3:9.1f} {(b - a) / 1e3:8.1f} q{q} {n}")


if __name__ == "__main__":
    main()
