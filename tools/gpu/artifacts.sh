# Round artifacts for one config: bench (+CPU baseline for C2), rocprofv3 kernel stats, and
# FETCH_SIZE / WRITE_SIZE passes.  usage: bash tools/gpu/artifacts.sh TAG CONFIG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFG=$2
O=gpurun_out/art_$TAG
mkdir -p $O
EXTRA=""; [ "$CFG" != "C2" ] && EXTRA="--no-cpu-baseline"
timeout -k 10 400 python bench.py --config $CFG $EXTRA > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --config $CFG --no-cpu-baseline > $O/stats.log 2>&1 || { tail -30 $O/stats.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py --config $CFG --steps 3 --warmup 2 --no-cpu-baseline > $O/fetch.log 2>&1 || { tail -30 $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python bench.py --config $CFG --steps 3 --warmup 2 --no-cpu-baseline > $O/write.log 2>&1 || { tail -30 $O/write.log; exit 1; }
python tools/pmc_summary.py $O/fetch $O/write $O/pmc.json | head -8
cut -c1-400 $O/bench.json
