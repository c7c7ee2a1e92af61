#!/bin/bash
# Round 4: MX depthwise-LN epilogue + encoder suites, then C5 / C3 / C4 benches on the current tree
set -o pipefail
O=gpurun_out/r4c5c3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mx_gpu.py tests/test_dwconv_cp_gpu.py tests/test_encoder_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in C5 C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 60 --warmup 10 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d.get('roofline',{}).get('kernel'), d.get('roofline',{}).get('frac'))"
done
