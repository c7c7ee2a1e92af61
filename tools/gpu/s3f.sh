set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
IMGCAP_GEMM256=7 timeout -k 10 300 python tools/gemm_census.py C2 > gpurun_out/census_C2_m7.txt 2>&1 || { tail -20 gpurun_out/census_C2_m7.txt; exit 1; }
sed -n 2,3p gpurun_out/census_C2_m7.txt
bash tools/gpu/artifacts.sh r02c2 C2 r02 || exit 1
bash tools/gpu/sqpass.sh C2 r02 || exit 1
