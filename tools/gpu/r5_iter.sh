#!/bin/bash
# Round 5 GEMM iteration: parity suite of the stream-tile kernel, phase stamps (diag library),
# shape sweep
set -o pipefail
O=gpurun_out/r5iter; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pt_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in ${CFGS:-2 4}; do
  timeout -k 10 120 python -u tools/pt_stamps.py $c >> $O/stamps.txt 2>&1 || { cat $O/stamps.txt; exit 1; }
done
grep -v amdgpu.ids $O/stamps.txt | sed 's/(p10.*//'
timeout -k 10 300 python -u tools/pt_bench.py 20 > $O/bench.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/bench.txt; exit $rc
