#!/bin/bash
# Round-6 final tree after the ws rule change: C2 and C3 artifacts (SQ for both), the full GPU suite, smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
SQ=1 bash tools/gpu/r6_art.sh C2 C3 || exit 1
O=gpurun_out/r6final2; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -n "FAILED" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
