# same-box A/B of an alternative library (IMGCAP_LIB) on C3/C4, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in "" $1 "" $1; do
  for c in C3 C4; do
    IMGCAP_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "lib=${lib:-default} $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:3], d["value"], d["ms_per_step"])')"
  done
done
