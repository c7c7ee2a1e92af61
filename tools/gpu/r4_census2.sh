#!/bin/bash
# Per-GEMM census (ours vs hipBLASLt) at C3 / C4 / C2 on the current tree.
set -o pipefail
O=gpurun_out/r4census2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_census.py C3 > $O/C3.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_census.py C4 > $O/C4.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_census.py C2 > $O/C2.txt 2>&1
