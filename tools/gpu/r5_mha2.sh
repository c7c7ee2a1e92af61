#!/bin/bash
# the LSTM checkpoint test (the scratch race of the two-pass colsum) first, then the MHA suites
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5mha2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_checkpoint_gpu.py tests/test_kernels_gpu.py > $O/t1.log 2>&1; rc=$?; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r5_mha.sh
