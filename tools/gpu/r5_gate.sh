#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5gate; rm -rf $O; mkdir -p $O
for order in afirst bfirst; do for na in 30 100; do kind=sleep; hq=4
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/t$order$na -o run -- python tools/probe/graph_gate.py $na $kind $order > $O/log$kind.txt 2>&1 || { tail -5 $O/log$kind.txt; exit 1; }
  python - $na $order $na <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/r5gate/t{sys.argv[2]}{sys.argv[3]}/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-(int(sys.argv[1]) + 6):]   # the last replay: 1 add + NA sleeps + 5 muls
t0 = int(rows[0]["Start_Timestamp"])
small = lambda r: "sleep" in r["Kernel_Name"].lower() or "spin" in r["Kernel_Name"].lower()
# branch A = the NA kernels of the side queue; B = the rest
qa = max(set(r.get("Queue_Id", "") for r in rows), key=lambda q: sum(1 for r in rows if r.get("Queue_Id", "") == q))
sleeps = [r for r in rows if r.get("Queue_Id", "") == qa]
others = [r for r in rows if r not in sleeps]
for r in others:
    st = int(r["Start_Timestamp"])
    before = sum(1 for s in sleeps if int(s["End_Timestamp"]) <= st)
    print(f"order={sys.argv[2]} NA={sys.argv[1]} {r['Kernel_Name'][:40]:40s} q{r.get('Queue_Id','?')} start {(st - t0) / 1e3:8.1f} us, sleeps done before it: {before}")
PY
done; done
