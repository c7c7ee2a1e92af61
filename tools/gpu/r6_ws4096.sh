#!/bin/bash
# ws by-shape rule down to M >= 4096 at K = 384 (C2's stage-3 fc1): old / new product libraries
# swapped in this box's copy, C2 / C3 alternating; then the stream-tile table (pt_bench) on the new.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ws4096
mkdir -p $O
LIB=imagecaptioningconvnext_amd/libimgcap_hip.so
cp build/libimgcap_hip_new.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_ws_gpu.py tests/test_encoder_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for cfg in C2; do
  for v in old new old new; do
    cp build/libimgcap_hip_$v.so $LIB
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 200 > $O/${cfg}_$v.log 2>&1 || { tail -20 $O/${cfg}_$v.log; exit 1; }
    echo "$cfg $v $(tail -1 $O/${cfg}_$v.log | cut -c1-100)"
  done
done
cp build/libimgcap_hip_new.so $LIB
timeout -k 10 300 python tools/pt_bench.py 20 > $O/pt.txt 2>&1 || { tail -20 $O/pt.txt; exit 1; }
cat $O/pt.txt | grep -v amdgpu
