#!/bin/bash
# round 6: engine-vs-emulating-oracle diagnostics, then the new tests (not the headline bf16 ones)
set -o pipefail
O=gpurun_out/r6b; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u tools/dec_emu_diag.py 64 768 1 > $O/diag1.log 2>&1; rc=$?; tail -40 $O/diag1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_headline_lstm_bf16_gpu.py tests/test_rccl_gpu.py \
  tests/test_stream_hazards_gpu.py "tests/test_transformer_gpu.py::test_mha_kernel_fwd_bwd" \
  tests/test_encoder_gpu.py tests/test_gemm_pt_gpu.py > $O/new.log 2>&1; rc=$?
tail -3 $O/new.log
exit $rc
