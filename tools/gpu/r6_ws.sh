#!/bin/bash
# round 6: weight-stationary short-K GEMM -- parity tests, then timings against the current plan
set -o pipefail
O=gpurun_out/r6ws; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_ws_gpu.py > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/ws_bench.py 20 > $O/bench.txt 2>&1; rc=$?; cat $O/bench.txt; exit $rc
