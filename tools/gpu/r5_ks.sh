#!/bin/bash
set -o pipefail
O=gpurun_out/r5ks; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pt_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MODES="4 7" bash tools/gpu/r5_sq.sh || exit 1
timeout -k 10 300 python -u tools/pt_bench.py 20 > $O/bench.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/bench.txt; exit $rc
