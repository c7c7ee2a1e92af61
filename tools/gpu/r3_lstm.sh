# round 3: granule hand-offs in the persistent LSTM forward -- parity, A/B of the h hand-off
# (granules vs write-through + flags) and of the poll throttle, stamps, C2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3lstm
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lstm_gpu.py -k "persist" > $O/t.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
IMGCAP_LSTM_HGRAN=0 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lstm_gpu.py -k "persist" > $O/t0.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t0.log | head -20; tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
for cfg in "0 0" "1 0"; do
  set -- $cfg
  IMGCAP_MB_B=32 IMGCAP_LSTM_GROUPS=1 IMGCAP_LSTM_HGRAN=$1 IMGCAP_LSTM_POLL_SLEEP=$2 IMGCAP_LSTM_STAMPS=1 timeout -k 10 120 python -u tools/microbench.py lstm > $O/mb_h$1_s$2.log 2>&1 || { tail -20 $O/mb_h$1_s$2.log; exit 1; }
  echo "== hgran=$1 sleep=$2"; grep -E "fwd recurrence B|U/G block|R block 0, |cross: G" $O/mb_h$1_s$2.log
done
for cfg in "0 0" "1 0"; do
  set -- $cfg
  IMGCAP_LSTM_HGRAN=$1 IMGCAP_LSTM_POLL_SLEEP=$2 timeout -k 10 300 python -u bench.py --config C2 --steps 100 --no-cpu-baseline > $O/c2_h$1_s$2.log 2>&1 || { tail -30 $O/c2_h$1_s$2.log; exit 1; }
  echo "== C2 hgran=$1 sleep=$2: $(tail -1 $O/c2_h$1_s$2.log | cut -c1-120)"
done
