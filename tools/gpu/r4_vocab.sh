#!/bin/bash
# vocab projection (3328 x 9490 x 512) and the decoder shapes under each tile plan, 16-byte output rows
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4vocab; mkdir -p $O
MODES=-1,4,6,7 timeout -k 10 300 python -u tools/gemm_modes.py > $O/modes.txt 2>&1 && grep -v amdgpu.ids $O/modes.txt &&
IMGCAP_GEMM_PT=1 MODES=-1 timeout -k 10 300 python -u tools/gemm_modes.py > $O/pt.txt 2>&1 && grep -v amdgpu.ids $O/pt.txt
