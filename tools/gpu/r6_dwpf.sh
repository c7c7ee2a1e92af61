#!/bin/bash
# dwconv7_cp rows of loads in flight (IMGCAP_DW_CP_PF 1/2/3): parity, per-launch time, C3 A/B.
# (The PF variants were slower and removed; the switch no longer exists.)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6dwpf
mkdir -p $O
for pf in 2 3; do
  IMGCAP_DW_CP_PF=$pf timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dwconv_cp_gpu.py > $O/tests$pf.txt 2>&1 || { tail -20 $O/tests$pf.txt; exit 1; }
  tail -1 $O/tests$pf.txt
done
for pf in 1 2 3 1 2 3; do
  IMGCAP_DW_CP_PF=$pf timeout -k 10 120 python tools/dw_cp_bench.py >> $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
done
grep PF= $O/bench.txt
for pf in 1 3 1 3; do
  IMGCAP_DW_CP_PF=$pf timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline --steps 100 > $O/c3_$pf.log 2>&1 || { tail -20 $O/c3_$pf.log; exit 1; }
  echo "PF=$pf $(tail -1 $O/c3_$pf.log | cut -c1-110)"
done
