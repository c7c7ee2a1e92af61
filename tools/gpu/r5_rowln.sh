#!/bin/bash
# fused GEMM + LayerNorm: kernel tests first, then the decoder suites, microbench and bench
set -o pipefail
O=gpurun_out/r5rowln; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_add_ln or gemm_ln_bwd" > $O/t0.log 2>&1; rc=$?; tail -3 $O/t0.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" $O/t0.log | head; exit $rc; }
timeout -k 10 120 python -u tools/chain_bench.py 20 > $O/chain.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/chain.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transformer_gpu.py tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py tests/test_headline_bf16_gpu.py tests/test_attvis_gpu.py tests/test_beam_gpu.py tests/test_greedy_gpu.py tests/test_checkpoint_gpu.py tests/test_testpy_gpu.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -n "Error\|assert" $O/tests.log | head -20; exit 1; }
for c in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b_$c.txt 2>$O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  echo "$c $(python -c "import json; d=json.loads(open('$O/b_$c.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
