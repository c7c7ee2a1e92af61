# forward attention channel-chunk sweep (IMGCAP_LSTM_ATT_YS): LSTM parity tests at each chunking,
# the recurrence microbench and the C2 bench.  usage: bash tools/gpu/att_ys.sh [ys...]
set -o pipefail
cd $GRAFT_REPO_ROOT
for ys in ${@:-1 2 3 4 6}; do
  IMGCAP_LSTM_ATT_YS=$ys timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lstm_gpu.py tests/test_greedy_gpu.py tests/test_beam_gpu.py > gpurun_out/ys_t.log 2>&1 || { tail -30 gpurun_out/ys_t.log; exit 1; }
  echo "ys=$ys tests: $(tail -1 gpurun_out/ys_t.log)"
  IMGCAP_LSTM_ATT_YS=$ys timeout -k 10 120 python tools/microbench.py lstm 2>&1 | grep "recurrence" || exit 1
  IMGCAP_LSTM_ATT_YS=$ys timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ys_b.log 2>&1 || { tail -20 gpurun_out/ys_b.log; exit 1; }
  echo "ys=$ys C2 $(tail -1 gpurun_out/ys_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
