#!/bin/bash
# the by-shape stream-tile plan as default: parity, census, C3 / C4 bench A/B (plan vs LDS-staged only)
set -o pipefail
O=gpurun_out/r5plan; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_pt_gpu.py tests/test_headline_bf16_gpu.py > $O/tests.log 2>&1; rc=$?
tail -30 $O/tests.log
[ $rc -le 1 ] || exit $rc
CFGS="C3 C4" PT_MODES="0 -1" bash tools/gpu/r5_census.sh | grep "step GEMM" || exit 1
for c in C3 C4; do
  for m in -1 0; do
    IMGCAP_GEMM_PT=$m timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b_${c}_$m.txt 2>$O/b_${c}_$m.err || { tail -20 $O/b_${c}_$m.err; exit 1; }
    echo "$c pt=$m $(python -c "import json,sys; d=json.loads(open('$O/b_${c}_$m.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
  done
done
