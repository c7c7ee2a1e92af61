set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "96,128,192" "96,128"; do
  for c in C2 C3; do
    IMGCAP_FUSED_MLP_C=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$v $c $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
