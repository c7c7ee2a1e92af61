#!/bin/bash
# clip + Adam captured in the pipelined graph: kernel + trainer parity, then C3 / C2 / C4 A/B
# (the in-graph Adam variant -- imgcap_clamp_adam_dyn, IMGCAP_ADAM_IN_GRAPH -- measured no gain and was
# removed; DESIGN 2b.  The script is kept as the record of the run.)
set -o pipefail
O=gpurun_out/r5adam; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "adam" tests/test_train_step_gpu.py tests/test_headline_bf16_gpu.py tests/test_transformer_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" $O/tests.log | head -20; exit 1; }
for r in 1 2; do
for c in C3 C2 C4; do
  for a in 1 0; do
    IMGCAP_ADAM_IN_GRAPH=$a timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
    echo "$c adam_in_graph=$a $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
  done
done
done
