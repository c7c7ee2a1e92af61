set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_s3c.log 2>&1 || { tail -30 gpurun_out/t_s3c.log; exit 1; }
tail -1 gpurun_out/t_s3c.log
for c in C2 C3; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${c}_s3c.log 2>&1 || { tail -30 gpurun_out/bench_${c}_s3c.log; exit 1; }
tail -1 gpurun_out/bench_${c}_s3c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['workload'][:3], d['value'], d['ms_per_step'], 'mfma', d['step_mfma_frac'], r['kernel'], r['frac'], r.get('sq'))"
done
timeout -k 10 300 python tools/gemm_census.py C2 > gpurun_out/census_C2_s3c.txt 2>&1 || { tail -20 gpurun_out/census_C2_s3c.txt; exit 1; }
sed -n 2,3p gpurun_out/census_C2_s3c.txt
