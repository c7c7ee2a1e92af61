#!/bin/bash
# Round 4: persistent-tile GEMM parity tests, then its shape sweep against the LDS-staged plan
# and hipBLASLt.
set -o pipefail
O=gpurun_out/r4pt; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pt_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/pt_bench.py 20 > $O/bench.txt 2>&1; rc=$?; cat $O/bench.txt; exit $rc
