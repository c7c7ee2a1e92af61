#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5seed; rm -rf $O; mkdir -p $O
for v in 1 0; do
  IMGCAP_PIPE_SEED_END=$v bash tools/gpu/r4_trace.sh C3 > $O/trace_$v.txt 2>&1 || { tail -20 $O/trace_$v.txt; exit 1; }
  echo "seed_end=$v"; grep -E "wall|queue [0-9]" $O/trace_$v.txt | head -4
  IMGCAP_PIPE_SEED_END=$v timeout -k 10 300 python -u bench.py --config C3 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "C3 seed_end=$v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
