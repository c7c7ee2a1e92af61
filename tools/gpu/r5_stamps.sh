#!/bin/bash
# Round 5: in-kernel phase stamps of the stream-tile GEMM (diagnostic library, built beforehand:
# make -C imagecaptioningconvnext_amd/csrc diag)
set -o pipefail
O=gpurun_out/r5stamps; mkdir -p $O
for c in ${CFGS:-2 4}; do
  timeout -k 10 120 python -u tools/pt_stamps.py $c >> $O/stamps.txt 2>&1 || { cat $O/stamps.txt; exit 1; }
done
grep -v amdgpu.ids $O/stamps.txt
