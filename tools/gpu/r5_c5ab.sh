#!/bin/bash
set -o pipefail
O=gpurun_out/r5c5ab; rm -rf $O; mkdir -p $O
for r in 1 2; do
for v in "" "IMGCAP_GEMM_PT=0" "IMGCAP_COLSUM=1"; do
  env $v timeout -k 10 300 python -u bench.py --config C5 --steps 60 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "C5 [$v] $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
done
