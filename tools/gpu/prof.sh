# usage: bash tools/gpu/prof.sh TAG CONFIG [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log
find gpurun_out/prof_$TAG -name "*kernel_stats.csv"
