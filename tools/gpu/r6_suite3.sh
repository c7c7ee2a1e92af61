#!/bin/bash
# round 6: full GPU suite + smoke (MHA probability-image swizzle, embedding chunks, nested-fork guard)
set -o pipefail
O=gpurun_out/r6suite3; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
