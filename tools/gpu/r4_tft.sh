#!/bin/bash
# fused Transformer loss-row prep (imgcap_tf_targets): kernel + trainer suites, then C3 / C4 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4tft; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k tf_targets tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py tests/test_transformer_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for cfg in C3 C4; do
  timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$cfg $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
