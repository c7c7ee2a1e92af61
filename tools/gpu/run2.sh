set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { tail -30 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python bench.py --config C3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || { tail -30 gpurun_out/prof_c3.log; exit 1; }
echo done
