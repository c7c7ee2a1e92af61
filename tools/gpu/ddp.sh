# trainer DDP paths (gloo, 2 ranks on the one GPU) + train-step tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train_step_gpu.py -k "bucketed or ddp2" > gpurun_out/ddp.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error" gpurun_out/ddp.log | tail -30
exit $rc
