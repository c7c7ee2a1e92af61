#!/bin/bash
# Embedding backward with 16-position chunks: kernel tests, C3 bench, kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6emb
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "embedding" tests/test_transformer_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2; do
timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > $O/bench$i.log 2>&1 || { tail -20 $O/bench$i.log; exit 1; }
tail -1 $O/bench$i.log | cut -c1-160
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --config C3 --no-cpu-baseline --steps 50 > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
rm -f $O/stats/run_kernel_trace.csv
grep -h "emb_" $O/stats/run_kernel_stats.csv | cut -c1-200
