#!/bin/bash
# hardware queues per process (GPU_MAX_HW_QUEUES; 4 on the box) against the pipelined graphs
set -o pipefail
O=gpurun_out/r5hwq; rm -rf $O; mkdir -p $O
for r in 1 2; do for c in C3 C2; do for q in 4 2 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "$c hwq=$q $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done; done; done
