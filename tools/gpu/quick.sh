# tests + C2/C3 benches (no CPU baseline). usage: bash tools/gpu/quick.sh TAG [configs...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
CFGS=${@:-C2 C3}
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
for c in $CFGS; do
timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${c}_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_${c}_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_${c}_$TAG.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['workload'][:3], d['value'], d['ms_per_step'], 'mfma', d['step_mfma_frac'], r['kernel'], r['frac'])"
done
