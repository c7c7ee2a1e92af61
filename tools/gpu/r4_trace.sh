#!/bin/bash
# Step timeline of a bench config (graph replays): rocprofv3 kernel trace -> tools/trace_path.py
# usage: bash tools/gpu/r4_trace.sh CFG [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=$1; shift
O=gpurun_out/trace_$CFG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python bench.py --config $CFG --steps 12 --warmup 3 --no-cpu-baseline --no-roofline "$@" > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
T=$(find $O/t -name '*kernel_trace.csv' | head -1)
python tools/trace_path.py $T --steps 2 --dump > $O/path.txt || exit 1
rm -f $T
head -60 $O/path.txt
