# round 3: LSTM / trainer GPU tests, then the C2 bench twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lstm_gpu.py tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py > $O/t.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config C2 --steps 100 --no-cpu-baseline --no-roofline > $O/c2_$i.log 2>&1 || { tail -30 $O/c2_$i.log; exit 1; }
  echo "C2 run $i: $(tail -1 $O/c2_$i.log | cut -c1-110)"
done
