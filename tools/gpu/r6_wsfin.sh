#!/bin/bash
# ws kernel after the GELU change and the variant move: its tests, the GEMM suites, a C3 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6wsfin
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_ws_gpu.py tests/test_gemm_pt_gpu.py tests/test_encoder_gpu.py tests/test_kernels_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
tail -1 $O/c3.log | cut -c1-110
