#!/bin/bash
# Round 5: stream-tile GEMM phase stamps with diagnostic switches (what bounds the k-step)
set -o pipefail
O=gpurun_out/r5dbg; rm -rf $O; mkdir -p $O
for d in 0 1 2 4 6; do
  for c in 2 4; do
    IMGCAP_PT_DBG=$d timeout -k 10 120 python -u tools/pt_stamps.py $c >> $O/stamps.txt 2>&1 || { cat $O/stamps.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/stamps.txt | sed 's/(p10.*//'
