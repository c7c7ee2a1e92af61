set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lstm_gpu.py tests/test_transformer_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_s3b.log 2>&1 || { tail -30 gpurun_out/t_s3b.log; exit 1; }
tail -1 gpurun_out/t_s3b.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_C2_s3b.log 2>&1 || { tail -30 gpurun_out/bench_C2_s3b.log; exit 1; }
tail -1 gpurun_out/bench_C2_s3b.log | cut -c1-400
bash tools/gpu/gemm_knobs.sh C2 0:2 1:2 0:3 1:3 0:4 1:4
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u tools/probe/cfg_diag.py C5 > gpurun_out/diag_c5_eager.log 2>&1 || { tail -30 gpurun_out/diag_c5_eager.log; exit 1; }
tail -3 gpurun_out/diag_c5_eager.log
