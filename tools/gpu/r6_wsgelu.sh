#!/bin/bash
# ws kernel GELU epilogue: polynomial erf (gelu_fast2) vs the sigmoid form (gelu_sig,
# IMGCAP_WS_GELU=sig): tests under the latter, per-launch time and C3 A/B on one box.
# (sig won and is the kernel's only form since; the switch is gone.)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6wsgelu
mkdir -p $O
IMGCAP_WS_GELU=sig timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_ws_gpu.py tests/test_encoder_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for g in poly sig; do
  IMGCAP_WS_GELU=$g WS_SHAPES="12544,1536,384,gelu;25088,1536,384,gelu" timeout -k 10 120 python tools/ws_bench.py 30 > $O/ws_$g.txt 2>&1 || { tail -20 $O/ws_$g.txt; exit 1; }
  echo "$g: $(grep custom $O/ws_$g.txt | tr '\n' ' ')"
done
for i in 1 2; do
  for g in poly sig; do
    IMGCAP_WS_GELU=$g timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > $O/c3_${g}_$i.log 2>&1 || { tail -20 $O/c3_${g}_$i.log; exit 1; }
    echo "$g $(tail -1 $O/c3_${g}_$i.log | cut -c1-100)"
  done
done
