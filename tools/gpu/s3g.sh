set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lstm_gpu.py > gpurun_out/s3g_t.log 2>&1 || { tail -20 gpurun_out/s3g_t.log; exit 1; }
tail -1 gpurun_out/s3g_t.log
IMGCAP_LSTM_STAMPS=1 timeout -k 10 120 python tools/microbench.py lstm 2>&1 | grep -E "bwd|recurrence:" || exit 1
timeout -k 10 240 python -u tools/probe/capture_bisect.py C4 split full2 > gpurun_out/bisect.log 2>&1; rc=$?
grep -v "^frame" gpurun_out/bisect.log | grep -v Warn | grep -E "^ok|bisect|Error" | head -12
exit $rc
