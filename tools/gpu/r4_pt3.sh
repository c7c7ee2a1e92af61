#!/bin/bash
# Round 4: persistent-tile GEMM with a branch-free k-step: parity tests, shape sweep vs the
# LDS-staged plan and hipBLASLt
set -o pipefail
O=gpurun_out/r4pt3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pt_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/pt_bench.py 20 > $O/bench.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/bench.txt; exit $rc
