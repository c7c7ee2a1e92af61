# kernel trace of a short bench run + one-step breakdown.  usage: bash tools/gpu/brk.sh TAG CFG [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/brk_${CFG}_$TAG -o run -- python bench.py --config $CFG --steps 6 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/brk_${CFG}_$TAG.log 2>&1 || { tail -30 gpurun_out/brk_${CFG}_$TAG.log; exit 1; }
python tools/step_breakdown.py $(find gpurun_out/brk_${CFG}_$TAG -name "*kernel_trace.csv" | head -1) 4 40 > gpurun_out/brk_${CFG}_$TAG.txt
head -45 gpurun_out/brk_${CFG}_$TAG.txt
