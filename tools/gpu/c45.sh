set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
for c in C4 C5; do
timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${c}_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_${c}_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_${c}_$TAG.log | cut -c1-400
done
