#!/bin/bash
set -o pipefail
O=gpurun_out/r5cs2; rm -rf $O; mkdir -p $O
timeout -k 10 120 python -u tools/colsum_bench.py 10 > $O/cs.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/cs.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/mha_bench.py 20 > $O/mha.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/mha.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/chain_bench.py 20 > $O/chain.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/chain.txt; exit $rc
