# Full GPU pass: parity tests, benches (C2 with CPU baseline, C3), rocprof kernel stats of C2.
# usage: bash tools/gpu/round.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_c2_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_c2_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_c2_$TAG.log
timeout -k 10 400 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c3_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_c3_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_c3_$TAG.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2_$TAG -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c2_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_c2_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_c2_$TAG.log
