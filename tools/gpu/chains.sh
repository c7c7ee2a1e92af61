set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_ch.log 2>&1 || { tail -40 gpurun_out/t_ch.log; exit 1; }
tail -1 gpurun_out/t_ch.log
for n in 1 2 4; do
  IMGCAP_LSTM_CHAINS=$n timeout -k 10 200 python tools/microbench.py lstm 2>&1 | grep recurrence
  IMGCAP_LSTM_CHAINS=$n timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "chains $n C2 $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
