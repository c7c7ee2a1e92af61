#!/bin/bash
# runtime flags against the graph-branch gate (tools/probe/graph_gate.py, A first, NA = 100)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5flags; rm -rf $O; mkdir -p $O
i=0
for f in "NONE=1" "DEBUG_CLR_MAX_BATCH_SIZE=1024" "DEBUG_CLR_MAX_BATCH_SIZE=4" "DEBUG_CLR_BATCH_CPU_SYNC_SIZE=1024" "DEBUG_CLR_BATCH_CPU_SYNC_SIZE=4" "ROC_SIGNAL_POOL_SIZE=8192" "ROC_AQL_QUEUE_SIZE=65536" "GPU_MAX_COMMAND_BUFFERS=256" "ROC_CPU_WAIT_FOR_SIGNAL=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  i=$((i+1))
  env $f timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/t$i -o run -- python tools/probe/graph_gate.py 100 sleep afirst > $O/log$i.txt 2>&1 || { echo "$f failed"; tail -5 $O/log$i.txt; continue; }
  python - $O/t$i "$f" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-106:]
t0 = int(rows[0]["Start_Timestamp"])
qa = max(set(r["Queue_Id"] for r in rows), key=lambda q: sum(1 for r in rows if r["Queue_Id"] == q))
others = [r for r in rows if r["Queue_Id"] != qa]
st = int(others[1]["Start_Timestamp"]) if len(others) > 1 else -1
print(f"{sys.argv[2]:40s} B start {(st - t0) / 1e3:8.1f} us; wall {(int(rows[-1]['End_Timestamp']) - t0) / 1e3:8.1f} us")
PY
  rm -rf $O/t$i
done
