# the whole -m gpu suite (log in gpurun_out/full_<tag>.log)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/full_$TAG.log 2>&1; rc=$?
tail -25 gpurun_out/full_$TAG.log
exit $rc
