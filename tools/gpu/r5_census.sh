#!/bin/bash
set -o pipefail
O=gpurun_out/r5census; rm -rf $O; mkdir -p $O
for c in ${CFGS:-C3 C4}; do
  timeout -k 10 400 python -u tools/gemm_census.py $c 10 > $O/$c.txt 2>&1 || { tail -30 $O/$c.txt; exit 1; }
  grep -v amdgpu.ids $O/$c.txt
done
