#!/bin/bash
# Round 4: multi-bucket DDP (per-layer decoder buckets, 25 MiB encoder buckets) on the GPU box,
# then the LDS-staged GEMM tile-plan sweep
set -o pipefail
O=gpurun_out/r4ddp; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train_step_gpu.py -k "ddp or bucketed or kernel_nodes" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -15
timeout -k 10 200 python -u tools/gemm_modes.py > $O/modes.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/modes.txt; exit $rc
