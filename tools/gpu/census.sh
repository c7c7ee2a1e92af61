set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in ${@:-C2 C3}; do
timeout -k 10 300 python tools/gemm_census.py $c > gpurun_out/census_$c.txt 2>&1 || { tail -20 gpurun_out/census_$c.txt; exit 1; }
head -25 gpurun_out/census_$c.txt
done
