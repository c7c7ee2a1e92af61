#!/bin/bash
# Round-4 baseline: the new gate / eval-after-fine-tune tests, per-GEMM census (ours vs
# hipBLASLt) at C3 / C4 and a short C3 bench.
set -o pipefail
O=gpurun_out/r4census; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_step_gpu.py -k "timeout_raises or eval_after" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python -u tools/gemm_census.py C3 > $O/C3.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_census.py C4 > $O/C4.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config C3 --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_C3.json 2> $O/bench_C3.err
