set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
IMGCAP_GEMM_GLDS=0 timeout -k 10 200 python tools/microbench.py gemm > gpurun_out/mb0.log 2>&1
IMGCAP_GEMM_GLDS=1 timeout -k 10 200 python tools/microbench.py gemm > gpurun_out/mb1.log 2>&1
paste -d'|' <(cut -c1-110 gpurun_out/mb0.log) <(cut -c80-110 gpurun_out/mb1.log) | grep -v amdgpu.ids
