#!/bin/bash
# weight-gradient GEMMs of the upper layers forked mid-backward: parity + C3 / C4 A/B
set -o pipefail
O=gpurun_out/r5mid; rm -rf $O; mkdir -p $O
IMGCAP_TF_MID_FORK=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_step_gpu.py tests/test_transformer_gpu.py tests/test_headline_bf16_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" $O/tests.log | head; exit 1; }
for r in 1 2; do
for c in C3 C4; do
  for m in -1 3 2; do
    IMGCAP_TF_MID_FORK=$m timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
    echo "$c mid=$m $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
  done
done
done
