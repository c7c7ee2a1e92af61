# GEMM-epilogue GELU (bf16 outputs -> gelu_sig): full GPU suite, GEMM census, C2-C4 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_census.py C3 > gpurun_out/census_c3.txt 2>&1 || { tail -20 gpurun_out/census_c3.txt; exit 1; }
head -2 gpurun_out/census_c3.txt
bash tools/gpu/quick.sh q7 C2 C3 C4
