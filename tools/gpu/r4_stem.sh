#!/bin/bash
# stem with two pixels per thread: encoder suites, then C3 / C4 benches and the stem's kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4stem; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_encoder_gpu.py tests/test_encoder_train_gpu.py tests/test_kernels_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for cfg in C3 C4; do
  timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$cfg $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
rm -f $O/stats/run_kernel_trace.csv
grep -i "stem_kernel" $O/stats/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
