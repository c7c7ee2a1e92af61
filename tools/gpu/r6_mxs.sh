#!/bin/bash
# MX GEMM with split remainder tiles: tests, microbench (split on / off), C5 bench A/B.
# (The variant measured here -- IMGCAP_MX_SPLIT, commit history of round 6 -- was slower and removed;
#  DESIGN §7.  Without it the script times the shipped kernel twice.)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6mxs
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mx_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 120 python tools/microbench.py mx > $O/mb_split.txt 2>&1 || { tail -20 $O/mb_split.txt; exit 1; }
IMGCAP_MX_SPLIT=0 timeout -k 10 120 python tools/microbench.py mx > $O/mb_nosplit.txt 2>&1 || { tail -20 $O/mb_nosplit.txt; exit 1; }
paste -d'|' $O/mb_nosplit.txt $O/mb_split.txt | grep -v amdgpu
for i in 1 2; do
  IMGCAP_MX_SPLIT=0 timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline --steps 100 > $O/c5_off$i.log 2>&1 || { tail -20 $O/c5_off$i.log; exit 1; }
  timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline --steps 100 > $O/c5_on$i.log 2>&1 || { tail -20 $O/c5_on$i.log; exit 1; }
  echo "off $(tail -1 $O/c5_off$i.log | cut -c1-120)"
  echo "on  $(tail -1 $O/c5_on$i.log | cut -c1-120)"
done
