set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 1 2 3; do
IMGCAP_GEMM256=$m timeout -k 10 300 python tools/gemm_census.py C3 > gpurun_out/census_C3_g$m.txt 2>&1 || { tail -5 gpurun_out/census_C3_g$m.txt; exit 1; }
sed -n 2,3p gpurun_out/census_C3_g$m.txt
done
timeout -k 10 300 python tools/gemm_census.py C3 > gpurun_out/census_C3_def.txt 2>&1 || exit 1
sed -n 2,3p gpurun_out/census_C3_def.txt
