# Round artifacts for one config: FETCH_SIZE / WRITE_SIZE passes (-> profiles/<ROUND>_<CFG>_pmc.json,
# read by bench.py's roofline.traffic), then the bench line (+CPU baseline for C2) and the
# rocprofv3 kernel stats of the same command.  usage: bash tools/gpu/artifacts.sh TAG CONFIG [ROUND]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFG=$2; ROUND=${3:-r01}
O=gpurun_out/art_$TAG
mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py --config $CFG --steps 3 --warmup 2 --no-cpu-baseline > $O/fetch.log 2>&1 || { tail -30 $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python bench.py --config $CFG --steps 3 --warmup 2 --no-cpu-baseline > $O/write.log 2>&1 || { tail -30 $O/write.log; exit 1; }
python tools/pmc_summary.py $O/fetch $O/write $O/pmc.json | head -8
cp $O/pmc.json profiles/${ROUND}_${CFG}_pmc.json
EXTRA=""; [ "$CFG" != "C3" ] && EXTRA="--no-cpu-baseline"
timeout -k 10 400 python bench.py --config $CFG $EXTRA > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --config $CFG --no-cpu-baseline > $O/stats.log 2>&1 || { tail -30 $O/stats.log; exit 1; }
rm -f $O/stats/run_kernel_trace.csv  # per-dispatch trace: tens of MB (gpurun copies back <= 64 MiB)
cut -c1-600 $O/bench.json
