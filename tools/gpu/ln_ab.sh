# add+LayerNorm change: kernel + Transformer suites, then C3/C4 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py tests/test_train_step_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_ln.log 2>&1 || { tail -30 gpurun_out/t_ln.log; exit 1; }
tail -1 gpurun_out/t_ln.log
for c in C3 C4 C3 C4; do
timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:3], d['value'], d['ms_per_step'])"
done
