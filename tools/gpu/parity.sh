# parity suites touched this round, verbose with measured errors (-s)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_encoder_train_gpu.py > gpurun_out/parity.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|rel |vs |Error|assert" gpurun_out/parity.log | tail -60
exit $rc
