# LSTM row groups: persistent-recurrence tests, per-step microbench, C2 bench with 1 vs 2 groups
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lstm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/grp_t.log 2>&1 || { tail -40 gpurun_out/grp_t.log; exit 1; }
tail -2 gpurun_out/grp_t.log
IMGCAP_LSTM_STAMPS=1 timeout -k 10 300 python -u tools/microbench.py lstm > gpurun_out/grp_mb.log 2>&1 || { tail -20 gpurun_out/grp_mb.log; exit 1; }
cat gpurun_out/grp_mb.log
for G in 2 1; do
IMGCAP_LSTM_GROUPS=$G timeout -k 10 400 python bench.py --config C2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/grp_bench$G.log 2>&1 || { tail -30 gpurun_out/grp_bench$G.log; exit 1; }
echo "groups=$G"; tail -1 gpurun_out/grp_bench$G.log | cut -c1-200
done
