# C2 bench per LSTM row-group mode (IMGCAP_LSTM_GROUPS bit 0 fwd, bit 1 bwd) + persistent tests split
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
IMGCAP_LSTM_GROUPS=3 timeout -k 10 400 python -u -m pytest tests/test_lstm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/grp_t.log 2>&1 || { tail -40 gpurun_out/grp_t.log; exit 1; }
tail -1 gpurun_out/grp_t.log
for G in 0 1 2 3; do
for c in ${CFGS:-C2}; do
IMGCAP_LSTM_GROUPS=$G timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline $EXTRA > gpurun_out/grp_bench$G$c.log 2>&1 || { tail -30 gpurun_out/grp_bench$G$c.log; exit 1; }
echo "groups=$G $c $EXTRA $(tail -1 gpurun_out/grp_bench$G$c.log | cut -c60-140)"
done
done
