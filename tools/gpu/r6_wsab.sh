#!/bin/bash
# round 6: the weight-stationary plan in the step -- parity tests, then C3 / C4 / C2 with and without
# it, two alternating rounds (200 steps each, no roofline / cpu legs)
set -o pipefail
O=gpurun_out/r6wsab; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_ws_gpu.py tests/test_encoder_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --no-cpu-baseline --no-roofline --steps 200 --warmup 10"
for round in 1 2; do
  for cfg in C3 C4 C2; do
    for ws in 0 -1; do
      r=$(timeout -k 10 300 env IMGCAP_GEMM_WS=$ws $B --config $cfg 2>>$O/err.log | tail -1) || exit 1
      echo "$round $cfg ws=$ws $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
    done
  done
done
