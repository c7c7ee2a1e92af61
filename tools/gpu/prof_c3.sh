set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$TAG -o run -- python bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c3_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_c3_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_c3_$TAG.log | cut -c1-300
