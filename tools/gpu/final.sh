# what the driver runs at round end: GPU suite, smoke(), default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_final.log 2>&1 || { tail -40 gpurun_out/t_final.log; exit 1; }
tail -1 gpurun_out/t_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-400
