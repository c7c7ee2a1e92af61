#!/bin/bash
# GEMM epilogue GELU (LDS-staged tiles, stream tile, scalar tail): polynomial erf vs the sigmoid
# form, as two prebuilt product libraries swapped in this box's scratch copy of the tree;
# tests under the sigmoid form, then C3 / C4 / C5 on one box, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6geluab
mkdir -p $O
LIB=imagecaptioningconvnext_amd/libimgcap_hip.so
cp build/libimgcap_hip_sig.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_pt_gpu.py tests/test_encoder_gpu.py tests/test_encoder_train_gpu.py tests/test_mx_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for cfg in C4 C3 C5; do
  for v in poly sig poly sig; do
    cp build/libimgcap_hip_$v.so $LIB
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 100 > $O/${cfg}_$v.log 2>&1 || { tail -20 $O/${cfg}_$v.log; exit 1; }
    echo "$cfg $v $(tail -1 $O/${cfg}_$v.log | cut -c1-100)"
  done
done
