#!/bin/bash
# C2 row-group split of the persistent LSTM recurrences (IMGCAP_LSTM_GROUPS mask: bit 0 forward,
# bit 1 backward) against the trainer's default (forward only beside the pipelined encoder)
set -o pipefail
O=gpurun_out/r5lg; rm -rf $O; mkdir -p $O
for r in 1 2; do for v in default 0 1 2 3; do
  if [ $v = default ]; then unset IMGCAP_LSTM_GROUPS; else export IMGCAP_LSTM_GROUPS=$v; fi
  timeout -k 10 300 python -u bench.py --config C2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "C2 groups=$v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done; done
