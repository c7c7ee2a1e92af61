# round 3: the full GPU suite (one process), then smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { grep -E "FAIL|Error|error" $O/suite.log | head -20; tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --config C2 --steps 60 --no-cpu-baseline > $O/c2.log 2>&1 || { tail -30 $O/c2.log; exit 1; }
tail -1 $O/c2.log | cut -c1-400
