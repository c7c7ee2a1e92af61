#!/bin/bash
# depthwise taps staged in LDS: parity, microbench, C3 / C4 bench
# (the taps-in-LDS variant measured equal -- 50.6 vs 48.7 us at stage 1, C3 20.0k -- and was removed)
set -o pipefail
O=gpurun_out/r5dwlds; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_encoder_gpu.py tests/test_dwconv_cp_gpu.py tests/test_encoder_train_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" $O/tests.log | head; exit 1; }
timeout -k 10 200 python -u tools/microbench.py dw > $O/dw.txt 2>&1 && grep -v amdgpu.ids $O/dw.txt || exit 1
for r in 1 2; do for c in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "$c $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done; done
