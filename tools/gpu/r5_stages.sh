#!/bin/bash
# decoder-chain GEMM shapes under 2 / 3 / 4 stages of the 64x64 tile
set -o pipefail
O=gpurun_out/r5stages; rm -rf $O; mkdir -p $O
for s in 2 3 4 2; do
  IMGCAP_GLDS64_STAGES=$s timeout -k 10 200 python -u tools/dec_gemm_stages.py > $O/s$s.txt 2>&1 || { tail -20 $O/s$s.txt; exit 1; }
  cat $O/s$s.txt
done
