#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5gate; rm -rf $O; mkdir -p $O
for na in 100 30; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/t$na -o run -- python tools/probe/graph_gate.py $na > $O/log$na.txt 2>&1 || { tail -5 $O/log$na.txt; exit 1; }
  python - $na <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/r5gate/t{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-(int(sys.argv[1]) + 6):]   # the last replay: 1 add + NA sleeps + 5 muls
t0 = int(rows[0]["Start_Timestamp"])
sleeps = [r for r in rows if "sleep" in r["Kernel_Name"].lower() or "spin" in r["Kernel_Name"].lower()]
others = [r for r in rows if r not in sleeps]
for r in others:
    st = int(r["Start_Timestamp"])
    before = sum(1 for s in sleeps if int(s["End_Timestamp"]) <= st)
    print(f"NA={sys.argv[1]} {r['Kernel_Name'][:40]:40s} q{r.get('Queue_Id','?')} start {(st - t0) / 1e3:8.1f} us, sleeps done before it: {before}")
PY
done
