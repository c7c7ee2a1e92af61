set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
IMGCAP_GEMM256=5 timeout -k 10 300 python tools/gemm_census.py C2 > gpurun_out/census_C2_tiled.txt 2>&1 || { tail -20 gpurun_out/census_C2_tiled.txt; exit 1; }
sed -n 2,3p gpurun_out/census_C2_tiled.txt
timeout -k 10 300 python -u tools/probe/graph_call_diag.py C4 2 > gpurun_out/gcd_c4.log 2>&1 || { grep -v "^frame" gpurun_out/gcd_c4.log | tail -25; exit 1; }
tail -2 gpurun_out/gcd_c4.log
