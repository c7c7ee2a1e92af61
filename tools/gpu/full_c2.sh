# full GPU suite, then C2 bench (pipelined and sequential)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/full_t.log 2>&1 || { tail -40 gpurun_out/full_t.log; exit 1; }
tail -1 gpurun_out/full_t.log
for X in "" --no-pipeline; do
timeout -k 10 400 python bench.py --config C2 --steps 20 --warmup 5 --no-cpu-baseline $X > gpurun_out/full_b.log 2>&1 || { tail -30 gpurun_out/full_b.log; exit 1; }
echo "C2 $X $(tail -1 gpurun_out/full_b.log | cut -c60-150)"
done
