# LSTM forward change: parity (LSTM + trainer suites), phase stamps, C2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lstm_gpu.py tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py tests/test_greedy_gpu.py tests/test_beam_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_lstm.log 2>&1 || { tail -30 gpurun_out/t_lstm.log; exit 1; }
tail -1 gpurun_out/t_lstm.log
IMGCAP_LSTM_STAMPS=1 timeout -k 10 200 python tools/microbench.py lstm > gpurun_out/lstm_st.log 2>&1 || { tail -20 gpurun_out/lstm_st.log; exit 1; }
grep -E "recurrence|U/G block|R block|cross|sub-phases" gpurun_out/lstm_st.log | head -10
for i in 1 2; do
timeout -k 10 300 python bench.py --config C2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:3], d['value'], d['ms_per_step'])"
done
