#!/bin/bash
# Round 4: persistent-tile GEMM after the per-tile DMA sources + DMA pieces interleaved with the
# MFMA groups: parity tests, shape sweep vs the LDS-staged plan and hipBLASLt, stamps
set -o pipefail
O=gpurun_out/r4pt2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pt_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/pt_probe.py full > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
timeout -k 10 120 python -u tools/pt_stamps.py 2 > $O/stamps.txt 2>&1 || { cat $O/stamps.txt; exit 1; }
grep -v amdgpu.ids $O/stamps.txt
timeout -k 10 300 python -u tools/pt_bench.py 20 > $O/bench.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/bench.txt; exit $rc
