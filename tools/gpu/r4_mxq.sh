#!/bin/bash
# Round 4: register-resident MX quantiser, MX depthwise fusion off by default: MX + encoder-train
# suites, C5 A/B (IMGCAP_MX_DW=1 vs default) on one box
set -o pipefail
O=gpurun_out/r4mxq; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mx_gpu.py tests/test_encoder_train_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1 0; do
  IMGCAP_MX_DW=$v timeout -k 10 300 python -u bench.py --config C5 --steps 60 --warmup 10 --no-cpu-baseline > $O/bench_C5_$v.json 2> $O/bench_C5_$v.err || { tail -20 $O/bench_C5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C5_$v.json').read().strip().splitlines()[-1]); r=d['roofline']['ranked_us_per_step']; print('MX_DW=$v', d['value'], d['ms_per_step'], {k: r[k] for k in list(r)[:4]})"
done
