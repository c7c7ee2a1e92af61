#!/bin/bash
# Final-tree stability: C3 for 1,000 steps, C2 and C3 with COCO-like caption lengths.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6stab
mkdir -p $O
timeout -k 10 400 python bench.py --config C3 --no-cpu-baseline --steps 1000 > $O/c3_1000.log 2>&1 || { tail -20 $O/c3_1000.log; exit 1; }
echo "C3 1000 steps: $(tail -1 $O/c3_1000.log | cut -c1-110)"
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
echo "C2: $(tail -1 $O/c2.log | cut -c1-110)"
timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline --lengths coco > $O/c3_coco.log 2>&1 || { tail -20 $O/c3_coco.log; exit 1; }
echo "C3 coco: $(tail -1 $O/c3_coco.log | cut -c1-110)"
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --lengths coco > $O/c2_coco.log 2>&1 || { tail -20 $O/c2_coco.log; exit 1; }
echo "C2 coco: $(tail -1 $O/c2_coco.log | cut -c1-110)"
