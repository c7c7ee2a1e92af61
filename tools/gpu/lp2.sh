# persistent LSTM forward with 1 / 2 concurrent row chains (each its own persistent launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in 1 2; do
IMGCAP_LSTM_CHAINS=$c timeout -k 10 120 python tools/microbench.py lstm 2>&1 | grep recurrence
IMGCAP_LSTM_CHAINS=$c timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/lp2_b.log 2>&1 || { tail -20 gpurun_out/lp2_b.log; exit 1; }
tail -1 gpurun_out/lp2_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('chains $c C2', d['value'], d['ms_per_step'])"
done
