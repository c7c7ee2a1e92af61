#!/bin/bash
# Round 5: stream-tile GEMM (csrc/gemm_pt.h) -- parity suite, then the shape sweep against the
# LDS-staged plan and hipBLASLt; the bf16 headline-configuration parity test
set -o pipefail
O=gpurun_out/r5st; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pt_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/pt_bench.py 20 > $O/bench.txt 2>&1 || { cat $O/bench.txt; exit 1; }
grep -v amdgpu.ids $O/bench.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_headline_bf16_gpu.py > $O/headline.log 2>&1; rc=$?; tail -30 $O/headline.log; exit $rc
