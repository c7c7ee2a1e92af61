"""Per-step kernel breakdown of ONE timed train step from a rocprofv3 kernel_trace.csv.

    python tools/step_breakdown.py TRACE.csv [step_index] [top]

Steps are delimited by the clamp_adam kernel (one launch per step); the window between the
(step_index)-th and (step_index+1)-th Adam launch is one full step (graph replay + Adam)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "clamp_adam" in r["Kernel_Name"]]
a, b = adam[k - 1], adam[k]
win = rows[a + 1:b + 1]
t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
busy = collections.defaultdict(float)
cnt = collections.Counter()


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "")
    return n[:90]


for r in win:
    n = short(r["Kernel_Name"])
    busy[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[n] += 1
tot = sum(busy.values())
print(f"step wall {(t1 - t0) / 1e3:.1f} us, kernel busy {tot:.1f} us, launches {len(win)}, "
      f"gaps {(t1 - t0) / 1e3 - tot:.1f} us")
for n, v in sorted(busy.items(), key=lambda x: -x[1])[:top]:
    print(f"{v:9.1f} us {cnt[n]:5d}x avg {v / cnt[n]:7.2f}  {n}")
