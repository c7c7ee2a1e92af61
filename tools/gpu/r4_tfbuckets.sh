#!/bin/bash
# Transformer length buckets: trainer suites (incl. the bucket parity test), then C3 / C4 with
# COCO-like caption lengths, buckets on / off, and the default full-length C3 line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4tfb; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in C3 C4; do for nb in "" "--no-len-buckets"; do
  timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --lengths coco $nb > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$cfg coco $nb $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
timeout -k 10 200 python bench.py --config C3 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
echo "C3 full $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
