#!/bin/bash
# Round 4: vectorised LN + patchify (tests + microbench), then the MX / encoder suites and the
# C5 / C3 / C4 benches on the current tree
set -o pipefail
O=gpurun_out/r4lnp; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "patchify" tests/test_encoder_train_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/lnp_bench.py > $O/lnp.txt 2>&1 || { cat $O/lnp.txt; exit 1; }
grep -v amdgpu.ids $O/lnp.txt
bash tools/gpu/r4_c5c3.sh
