# round 3: per-step timeline of the C2 bench (kernel trace) -> critical path of the pipelined step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3trace
mkdir -p $O
CFG=${1:-C2}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$CFG -o run -- python bench.py --config $CFG --steps 12 --warmup 4 --no-cpu-baseline --no-roofline > $O/${CFG}_bench.log 2>&1 || { tail -20 $O/${CFG}_bench.log; exit 1; }
f=$(find $O/$CFG -name "*kernel_trace.csv" | head -1)
python tools/trace_path.py $f --steps 2 > $O/${CFG}_path.txt && head -70 $O/${CFG}_path.txt
python tools/trace_path.py $f --steps 1 --dump > $O/${CFG}_dump.txt
rm -f $f
