# persistent LSTM forward: parity tests, recurrence microbench (+ phase stamps), C2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lstm_gpu.py > gpurun_out/lp_t.log 2>&1; rc=$?
tail -12 gpurun_out/lp_t.log
[ $rc -ne 0 ] && exit $rc
IMGCAP_LSTM_STAMPS=1 timeout -k 10 120 python tools/microbench.py lstm 2>&1 | tail -8
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/lp_b.log 2>&1 || { tail -20 gpurun_out/lp_b.log; exit 1; }
tail -1 gpurun_out/lp_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['ms_per_step'])"
