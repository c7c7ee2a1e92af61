#!/bin/bash
# round 6: ws kernel -- software-pipelined form vs the lockstep form
set -o pipefail
O=gpurun_out/r6ws3; rm -rf $O; mkdir -p $O
S="1280,1536,384,gelu;5120,1536,384,gelu;12544,1536,384,gelu;25088,1536,384,gelu;50176,192,384,bias;3328,1536,512,bias;6272,2048,512,gelu;3136,6144,512,bias"
timeout -k 10 200 env IMGCAP_WS_PIPE=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_ws_gpu.py > $O/tests_pipe.log 2>&1; rc=$?; tail -2 $O/tests_pipe.log; [ $rc -eq 0 ] || exit $rc
for v in "IMGCAP_WS_STG=1" "IMGCAP_WS_PIPE=1"; do
  echo "== $v"; timeout -k 10 300 env WS_SHAPES="$S" $v python -u tools/ws_bench.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done
