# fused MLP kernel bench + MLP/encoder parity tests only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cd tools/kbench
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize -munsafe-fp-atomics $MLPFLAGS mlp_bench.hip -o /tmp/mlp_res 2>/dev/null || exit 1
timeout -k 5 60 /tmp/mlp_res || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_encoder_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_mlp.log 2>&1 || { tail -30 gpurun_out/t_mlp.log; exit 1; }
tail -1 gpurun_out/t_mlp.log
