#!/bin/bash
# two-graph pipelined step (encoder graph on its own, optionally CU-masked, stream): parity, C3 A/B, trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5g2; rm -rf $O; mkdir -p $O
IMGCAP_PIPE_GRAPHS=2 IMGCAP_ENC_CUS=192 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_step_gpu.py -k "pipelined" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" $O/tests.log | head; exit 1; }
for cus in 0 224 192 160; do
  IMGCAP_PIPE_GRAPHS=2 IMGCAP_ENC_CUS=$cus timeout -k 10 300 python -u bench.py --config C3 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "C3 graphs2 cus=$cus $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
timeout -k 10 300 python -u bench.py --config C3 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
echo "C3 one graph $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
IMGCAP_PIPE_GRAPHS=2 IMGCAP_ENC_CUS=192 bash tools/gpu/r4_trace.sh C3 > $O/trace.txt 2>&1 || { tail -5 $O/trace.txt; exit 1; }
grep -E "wall|queue [0-9]" $O/trace.txt | head -5
