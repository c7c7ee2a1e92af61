#!/bin/bash
# round 6: engine vs emulating oracle with the engine's operand precisions, then the headline tests
set -o pipefail
O=gpurun_out/r6c; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u tools/dec_emu_diag.py 64 768 1 > $O/diag1.log 2>&1; rc=$?; tail -42 $O/diag1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_headline_bf16_gpu.py \
  > $O/headline.log 2>&1; rc=$?
grep -A13 "^\[B=" $O/headline.log | head -80; tail -3 $O/headline.log
exit $rc
