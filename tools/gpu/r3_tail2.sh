# round 3: LSTM backward tail -- bias column sums beside the grouped GEMMs, optional inline Adam
# with the fc range after the backward recurrence: LSTM / trainer suites (inline Adam on and off),
# then C2 same-box A/B (default, IMGCAP_LSTM_CB_SIDE=0, IMGCAP_INLINE_ADAM=1), two rounds
# (IMGCAP_LSTM_CB_SIDE was a knob of the measured variant; removed after the A/B, so "cbmain" is now the default path)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tail2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_lstm_gpu.py tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py tests/test_checkpoint_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
IMGCAP_INLINE_ADAM=1 timeout -k 10 300 python -u -m pytest tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_inline.log 2>&1 || { tail -40 $O/test_inline.log; exit 1; }
tail -1 $O/test_inline.log
for i in 1 2; do
  for v in "base:" "cbmain:IMGCAP_LSTM_CB_SIDE=0" "inline:IMGCAP_INLINE_ADAM=1"; do
    n=${v%%:*}; e=${v#*:}
    env $e timeout -k 10 300 python bench.py --no-roofline --no-cpu-baseline > $O/${n}_$i.log 2>&1 || { tail -20 $O/${n}_$i.log; exit 1; }
    echo "$n $i: $(tail -1 $O/${n}_$i.log | cut -c1-120)"
  done
done
