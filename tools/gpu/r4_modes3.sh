#!/bin/bash
# 128x128 (mode 4) and 64x64 (mode 6) LDS-DMA tiles with 2 / 3 / 4 stages at the step's shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4modes3; mkdir -p $O
for s in 2 3 4; do
  IMGCAP_GLDS_STAGES=$s IMGCAP_GLDS64_STAGES=$s MODES=-1,4,6 timeout -k 10 300 python -u tools/gemm_modes.py > $O/s$s.txt 2>&1 || { tail -5 $O/s$s.txt; exit 1; }
  echo "stages=$s"; grep -v amdgpu.ids $O/s$s.txt
done
