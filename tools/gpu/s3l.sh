set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/t_s3l.log 2>&1 || { tail -30 gpurun_out/t_s3l.log; exit 1; }
tail -1 gpurun_out/t_s3l.log
for c in C2 C3; do bash tools/gpu/artifacts.sh r02_$c $c r02 || exit 1; done
