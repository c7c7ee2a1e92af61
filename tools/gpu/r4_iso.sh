#!/bin/bash
# Round 4: isolated timings of the attention, depthwise, MX and LN+depthwise kernels
set -o pipefail
O=gpurun_out/r4iso; mkdir -p $O
export TMPDIR=/tmp
for w in mha dw mx; do
  timeout -k 10 200 python -u tools/microbench.py $w > $O/$w.txt 2>&1 || { cat $O/$w.txt; exit 1; }
  grep -v amdgpu.ids $O/$w.txt
done
timeout -k 10 200 python -u tools/dw_ln_bench.py > $O/dwln.txt 2>&1 || { cat $O/dwln.txt; exit 1; }
grep -v amdgpu.ids $O/dwln.txt
