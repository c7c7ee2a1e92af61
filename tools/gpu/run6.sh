set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/t_run6.log 2>&1 || { tail -40 gpurun_out/t_run6.log; exit 1; }
tail -1 gpurun_out/t_run6.log
timeout -k 10 300 python tools/microbench.py lstm > gpurun_out/mb_lstm.log 2>&1 || { tail -20 gpurun_out/mb_lstm.log; exit 1; }
grep lstm gpurun_out/mb_lstm.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || { tail -30 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log
timeout -k 10 400 python bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { tail -30 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
