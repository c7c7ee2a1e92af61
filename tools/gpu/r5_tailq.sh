#!/bin/bash
# (IMGCAP_TAIL_ON_ENC was an experiment switch, measured 1-2 % slower and removed -- DESIGN 2b)
# the Transformer backward's tail column sums on the encoder branch's stream (one queue fewer)
set -o pipefail
O=gpurun_out/r5tailq; rm -rf $O; mkdir -p $O
for r in 1 2; do for c in C3 C4; do for v in 1 0; do
  IMGCAP_TAIL_ON_ENC=$v timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "$c tail_on_enc=$v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done; done; done
