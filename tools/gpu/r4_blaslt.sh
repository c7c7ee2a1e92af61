#!/bin/bash
# Round 4: the hipBLASLt kernels (names = macro tile, wave tiling, staging) torch.matmul picks at
# the encoder shapes, from a kernel trace
set -o pipefail
O=gpurun_out/r4blaslt; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/probe/blaslt_names.py > $GRAFT_REPO_ROOT/$O/log.txt 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/log.txt; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -1)
cut -c1-400 $f | head -20
