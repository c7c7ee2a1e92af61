# A/B of an alternative library build (IMGCAP_LIB): GEMM parity tests on it, GEMM census + C2/C3
# bench lines for both.  usage: bash tools/gpu/ab_lib.sh ALT_SO
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=$1
IMGCAP_LIB=$ALT timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t_alt.log 2>&1 || { tail -30 gpurun_out/t_alt.log; exit 1; }
tail -1 gpurun_out/t_alt.log
for lib in "" $ALT; do
  IMGCAP_LIB=$lib timeout -k 10 300 python tools/gemm_census.py C2 > gpurun_out/census_ab.txt 2>&1 || { tail -20 gpurun_out/census_ab.txt; exit 1; }
  echo "lib=${lib:-default}"; head -2 gpurun_out/census_ab.txt
  for c in C2 C3; do
    IMGCAP_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['workload'][:3], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['avg_launch_us'])"
  done
done
