# round 3: one GPU test file / selection (arguments: pytest node ids)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3one
IMGCAP_GRAD_REPORT=1 timeout -k 10 600 python -u -m pytest -s -v --timeout 300 --timeout-method thread "$@" > gpurun_out/r3one/t.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|grad rel" gpurun_out/r3one/t.log | head -40
exit $rc
