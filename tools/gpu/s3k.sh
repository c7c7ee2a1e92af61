set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config C5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_C5_s3k.log 2>&1 || { grep -v "^frame" gpurun_out/bench_C5_s3k.log | tail -8; exit 1; }
tail -1 gpurun_out/bench_C5_s3k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:3], d['value'], d['ms_per_step'])"
timeout -k 10 400 python -u -m pytest tests/test_train_step_gpu.py tests/test_encoder_train_gpu.py tests/test_trainer_fullsize_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/s3k_t.log 2>&1 || { tail -20 gpurun_out/s3k_t.log; exit 1; }
tail -1 gpurun_out/s3k_t.log
