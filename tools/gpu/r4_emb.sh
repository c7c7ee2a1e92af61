#!/bin/bash
# embedding gradient with batched row loads for long runs: kernel + trainer suites, then COCO-length
# C3 / C2 (buckets on / off) and the full-length C3 / C2 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4emb; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py tests/test_lstm_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in C3 C2 C4; do for nb in "" "--no-len-buckets"; do
  timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --lengths coco $nb > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$cfg coco $nb $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
for cfg in C3 C2; do
timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
echo "$cfg full $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
