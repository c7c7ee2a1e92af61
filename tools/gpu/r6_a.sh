#!/bin/bash
# round 6, first GPU pass: the new / tightened parity tests with their measured numbers (-s), then
# the whole GPU suite in one process
set -o pipefail
O=gpurun_out/r6a; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_headline_bf16_gpu.py tests/test_headline_lstm_bf16_gpu.py tests/test_rccl_gpu.py \
  tests/test_stream_hazards_gpu.py "tests/test_transformer_gpu.py::test_mha_kernel_fwd_bwd" \
  tests/test_encoder_gpu.py tests/test_gemm_pt_gpu.py > $O/new.log 2>&1; rc=$?
tail -3 $O/new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc2=$?
tail -3 $O/tests.log
exit $rc2
