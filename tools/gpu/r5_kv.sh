#!/bin/bash
# batched cross-attention K/V: chain microbench, transformer / trainer suites, C3 / C4 bench
set -o pipefail
O=gpurun_out/r5kv; rm -rf $O; mkdir -p $O
timeout -k 10 120 python -u tools/chain_bench.py 20 > $O/chain.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/chain.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transformer_gpu.py tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py tests/test_headline_bf16_gpu.py tests/test_attvis_gpu.py tests/test_beam_gpu.py tests/test_greedy_gpu.py tests/test_checkpoint_gpu.py > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -le 1 ] || exit $rc
for c in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b_$c.txt 2>$O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  echo "$c $(python -c "import json; d=json.loads(open('$O/b_$c.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
