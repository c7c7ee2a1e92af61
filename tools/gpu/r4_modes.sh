#!/bin/bash
# LDS-staged GEMM tile plans at the widest-gap shapes, 2 and 3 stages for the 128 tile
set -o pipefail
O=gpurun_out/r4modes; mkdir -p $O
timeout -k 10 200 python -u tools/gemm_modes.py > $O/s2.txt 2>&1 && grep -v amdgpu.ids $O/s2.txt &&
IMGCAP_GLDS_STAGES=3 timeout -k 10 200 python -u tools/gemm_modes.py > $O/s3.txt 2>&1 && grep -v amdgpu.ids $O/s3.txt
