# LSTM recurrence per-step time and stamps at several batch sizes: bash tools/gpu/lstm_b.sh B...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in "$@"; do
  IMGCAP_MB_B=$b IMGCAP_LSTM_STAMPS=1 timeout -k 10 300 python -u tools/microbench.py lstm > gpurun_out/lstm_b$b.log 2>&1 || { tail -20 gpurun_out/lstm_b$b.log; exit 1; }
  cat gpurun_out/lstm_b$b.log
done
