set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lstm_gpu.py > gpurun_out/s3j_t.log 2>&1 || { tail -20 gpurun_out/s3j_t.log; exit 1; }
tail -1 gpurun_out/s3j_t.log
IMGCAP_LSTM_STAMPS=1 timeout -k 10 120 python tools/microbench.py lstm 2>&1 | grep -E "bwd|recurrence:" || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_C2_s3j.log 2>&1 || { tail -20 gpurun_out/bench_C2_s3j.log; exit 1; }
tail -1 gpurun_out/bench_C2_s3j.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['ms_per_step'])"
bash tools/gpu/s3i.sh
