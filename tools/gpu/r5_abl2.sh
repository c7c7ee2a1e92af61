#!/bin/bash
set -o pipefail
O=gpurun_out/r5abl2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pt_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/pt_bench.py 20 > $O/bench.txt 2>&1 || { cat $O/bench.txt; exit 1; }
grep -v amdgpu.ids $O/bench.txt
for f in 1 0 1 0; do
  IMGCAP_TF_TAIL_FORK=$f timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 > $O/c3_fork$f.json 2> $O/c3_fork$f.err || { tail $O/c3_fork$f.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/c3_fork$f.json').read().strip().splitlines()[-1]); print('tail fork $f', d['value'], d['ms_per_step'])"
done
