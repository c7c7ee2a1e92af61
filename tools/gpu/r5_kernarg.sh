#!/bin/bash
# HIP_FORCE_DEV_KERNARG (kernel arguments in device memory) on the bench configs, alternating
# (first run: =1 vs =0 -- C3 20.35k vs 18.60k; this run: =1 vs unset)
set -o pipefail
O=gpurun_out/r5karg; rm -rf $O; mkdir -p $O
for r in 1 2; do for c in C3 C4; do for v in 1 unset; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "$c dev_kernarg=$v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done; done; done
