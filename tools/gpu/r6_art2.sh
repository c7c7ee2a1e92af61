#!/bin/bash
# Round-6 artifacts for C2 / C4 / C5 (+ SQ passes), then the decoder's small kernels in isolation
# (MHA self / cross fwd + bwd, dropout 0 / 0.1).  usage: bash tools/gpu/r6_art2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
SQ=1 bash tools/gpu/r6_art.sh C2 C4 C5 || exit 1
mkdir -p gpurun_out/r6mb
timeout -k 10 120 python tools/mha_bench.py 30 > gpurun_out/r6mb/mha.txt 2>&1 || { tail -20 gpurun_out/r6mb/mha.txt; exit 1; }
cat gpurun_out/r6mb/mha.txt
