#!/bin/bash
# C3 / C4: each library switch's alternate against the default, same box, two rounds
set -o pipefail
O=gpurun_out/r5knobs; rm -rf $O; mkdir -p $O
for r in 1 2; do for c in C3 C4; do
for v in "NONE=1" "IMGCAP_COLSUM=1" "IMGCAP_TF_TAIL_FORK=0" "IMGCAP_GEMM_ORDER=0" "IMGCAP_GEMM_ORDER=1" "IMGCAP_GEMM_PT=0" "IMGCAP_GEMM256=0" "IMGCAP_DW_CP_R=2"; do
  env $v timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "$c $v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done; done; done
