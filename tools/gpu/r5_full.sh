#!/bin/bash
# full GPU suite, microbenchmarks, C3 / C4 bench, C3 kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5full; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || { grep -n "Error\|assert" $O/tests.log | head -20; exit 1; }
timeout -k 10 120 python -u tools/mha_bench.py 20 > $O/mha.txt 2>&1 && grep -v amdgpu.ids $O/mha.txt || exit 1
timeout -k 10 120 python -u tools/chain_bench.py 20 > $O/chain.txt 2>&1 && grep -v amdgpu.ids $O/chain.txt | head -4 || exit 1
for c in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b_$c.txt 2>$O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  echo "$c $(python -c "import json; d=json.loads(open('$O/b_$c.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
