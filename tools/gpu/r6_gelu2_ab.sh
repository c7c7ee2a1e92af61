#!/bin/bash
# GEMM epilogue GELU: scalar sigmoid form (shipped) vs the packed-pair form (gelu_sig2), two prebuilt
# libraries swapped in this box's copy: kernel tests under the packed form, MX microbench, C4 / C5.
# (Measured equal; the packed form was not kept and the two libraries are no longer built.)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6gelu2
mkdir -p $O
LIB=imagecaptioningconvnext_amd/libimgcap_hip.so
cp build/libimgcap_hip_sig.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_mx_gpu.py tests/test_encoder_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in poly sig; do
  cp build/libimgcap_hip_$v.so $LIB
  timeout -k 10 120 python tools/microbench.py mx > $O/mx_$v.txt 2>&1 || { tail -20 $O/mx_$v.txt; exit 1; }
  echo "$v: $(grep 'GELU' $O/mx_$v.txt | tr '\n' ' ')"
done
for cfg in C4 C5; do
  for v in poly sig poly sig; do
    cp build/libimgcap_hip_$v.so $LIB
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 100 > $O/${cfg}_$v.log 2>&1 || { tail -20 $O/${cfg}_$v.log; exit 1; }
    echo "$cfg $v $(tail -1 $O/${cfg}_$v.log | cut -c1-100)"
  done
done
