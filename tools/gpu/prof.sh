# kernel trace of one config + per-step breakdown. usage: bash tools/gpu/prof.sh TAG CONFIG [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${CFG}_$TAG -o run -- python bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/prof_${CFG}_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_${CFG}_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_${CFG}_$TAG.log | cut -c1-300
python tools/step_breakdown.py $(find gpurun_out/prof_${CFG}_$TAG -name '*kernel_trace.csv' | head -1) 6 40 > gpurun_out/brk_${CFG}_$TAG.txt
