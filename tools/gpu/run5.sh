set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/t_run5.log 2>&1 || { tail -40 gpurun_out/t_run5.log; exit 1; }
tail -1 gpurun_out/t_run5.log
timeout -k 10 200 python tools/microbench.py misc > gpurun_out/mb.log 2>&1; grep -E "dwconv|add_ln|colsum" gpurun_out/mb.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || { tail -30 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log | cut -c1-200
timeout -k 10 300 python bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { tail -30 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log | cut -c1-200
