#!/bin/bash
# Stem with 4 patches per thread (IMGCAP_STEM_PX=4) vs 2: encoder tests, per-launch time, C3 / C2 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6stem
mkdir -p $O
for px in 2 4; do
  IMGCAP_STEM_PX=$px timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_encoder_gpu.py > $O/tests$px.txt 2>&1 || { tail -30 $O/tests$px.txt; exit 1; }
  echo "PX=$px tests: $(tail -1 $O/tests$px.txt)"
done
for px in 2 4 2 4; do
  IMGCAP_STEM_PX=$px timeout -k 10 120 python tools/stem_bench.py >> $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
done
grep PX= $O/bench.txt
for cfg in C3 C2; do
  for px in 2 4 2 4; do
    IMGCAP_STEM_PX=$px timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 100 > $O/${cfg}_$px.log 2>&1 || { tail -20 $O/${cfg}_$px.log; exit 1; }
    echo "$cfg PX=$px $(tail -1 $O/${cfg}_$px.log | cut -c1-100)"
  done
done
