# LSTM row-group masks at C2 (pipelined): IMGCAP_LSTM_GROUPS = 0 none, 1 fwd, 2 bwd, 3 both
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in ${MASKS:-1 3 2 0 1 3}; do  # measured: 1 (default) 12.30-12.46k, 2 12.39-12.55k, 3 12.06-12.14k, 0 12.14k
  IMGCAP_LSTM_GROUPS=$m timeout -k 10 300 python bench.py --config C2 --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "groups=$m $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
