set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/art_r02_C5
( while sleep 50; do echo "progress $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 500 python bench.py --config C5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/art_r02_C5/bench.log 2>&1 || { tail -20 gpurun_out/art_r02_C5/bench.log; exit 1; }
tail -1 gpurun_out/art_r02_C5/bench.log > gpurun_out/art_r02_C5/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/art_r02_C5/stats -o run -- python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/art_r02_C5/stats.log 2>&1 || { tail -20 gpurun_out/art_r02_C5/stats.log; exit 1; }
cut -c1-300 gpurun_out/art_r02_C5/bench.json
bash tools/gpu/sqpass.sh C3 r02 || exit 1
