#!/bin/bash
# Two more stream-tile shapes in the by-shape plan (Tiny stage-4 fc1, Base stage-3 fc1): tests under
# the new library, then old / new swapped in this box's copy, C4 / C3 alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ptrule
mkdir -p $O
LIB=imagecaptioningconvnext_amd/libimgcap_hip.so
cp build/libimgcap_hip_new.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_pt_gpu.py tests/test_encoder_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for cfg in C4 C3; do
  for v in old new old new; do
    cp build/libimgcap_hip_$v.so $LIB
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 200 > $O/${cfg}_$v.log 2>&1 || { tail -20 $O/${cfg}_$v.log; exit 1; }
    echo "$cfg $v $(tail -1 $O/${cfg}_$v.log | cut -c1-100)"
  done
done
