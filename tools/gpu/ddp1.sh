set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 150 python -u -m pytest -x -v -s --timeout 140 --timeout-method thread tests/test_train_step_gpu.py -k bucketed > gpurun_out/ddp1.log 2>&1
