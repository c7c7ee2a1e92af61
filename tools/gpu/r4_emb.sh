#!/bin/bash
# embedding gradient in aligned chunks + in-order combine: the whole GPU suite, then COCO-length and
# full-length benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4emb; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in C3 C2; do for nb in "" "--no-len-buckets"; do
  timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --lengths coco $nb > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$cfg coco $nb $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
for cfg in C3 C2 C4; do
timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
echo "$cfg full $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
