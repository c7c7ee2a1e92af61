# round 3: LSTM step with att1 / attn_reg / the embedding gradient off the critical path --
# the LSTM, trainer and checkpoint suites, then the default C2 bench (no roofline pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tail
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_lstm_gpu.py tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py tests/test_checkpoint_gpu.py tests/test_greedy_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-roofline --no-cpu-baseline > $O/bench$i.log 2>&1 || { tail -20 $O/bench$i.log; exit 1; }
  tail -1 $O/bench$i.log | cut -c1-200
done
