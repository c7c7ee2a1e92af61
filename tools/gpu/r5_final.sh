#!/bin/bash
# round-end check: full GPU suite (one process), smoke, default bench line
set -o pipefail
O=gpurun_out/r5final; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log | cut -c1-400; exit $rc
