set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/ -q -m gpu -x > gpurun_out/t_run1.log 2>&1 || { tail -30 gpurun_out/t_run1.log; exit 1; }
tail -2 gpurun_out/t_run1.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke1.log 2>&1 || { cat gpurun_out/smoke1.log; exit 1; }
cat gpurun_out/smoke1.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench1.log 2>&1 || { tail -30 gpurun_out/bench1.log; exit 1; }
tail -3 gpurun_out/bench1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 || { tail -30 gpurun_out/prof1.log; exit 1; }
find gpurun_out/prof1 -name "*stats*" | head
