# microbenchmarks + C3 profile. usage: bash tools/gpu/mb.sh TAG [groups...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
for g in "$@"; do
  timeout -k 10 300 python tools/microbench.py $g > gpurun_out/mb_${g}_$TAG.log 2>&1 || { tail -20 gpurun_out/mb_${g}_$TAG.log; exit 1; }
  cat gpurun_out/mb_${g}_$TAG.log
done
