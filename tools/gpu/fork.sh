# two-branch pipeline graph: encoder branch forked at the step start (default) vs after the
# decoder forward.  usage: bash tools/gpu/fork.sh [configs...]
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 env IMGCAP_PIPE_FORK=bwd python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_step_gpu.py > gpurun_out/fork_t.log 2>&1 || { tail -30 gpurun_out/fork_t.log; exit 1; }
echo "fork=bwd tests: $(tail -1 gpurun_out/fork_t.log)"
for c in ${@:-C2 C3}; do for f in start bwd start bwd; do
  IMGCAP_PIPE_FORK=$f timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/fk.log 2>&1 || { tail -20 gpurun_out/fk.log; exit 1; }
  echo "fork=$f $c $(tail -1 gpurun_out/fk.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
