#!/bin/bash
# GEMM tile plans (incl. the three 256x256 variants) at the C3/C4 encoder and decoder shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4modes2; mkdir -p $O
timeout -k 10 300 python -u tools/gemm_modes.py > $O/modes.txt 2>&1 && grep -v amdgpu.ids $O/modes.txt
