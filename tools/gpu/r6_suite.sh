#!/bin/bash
# round 6: full GPU suite (one process) + smoke
set -o pipefail
O=gpurun_out/r6suite; rm -rf $O; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc2=$?; tail -2 $O/smoke.log
exit $((rc + rc2))
