#!/bin/bash
# Round 4: register-resident bf16 attention: kernel + Transformer suites, isolated timing, C3 bench
set -o pipefail
O=gpurun_out/r4mha; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/microbench.py mha > $O/mha.txt 2>&1 || { cat $O/mha.txt; exit 1; }
grep -v amdgpu.ids $O/mha.txt
timeout -k 10 300 python -u bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/bench_C3.json 2> $O/bench_C3.err || { tail -20 $O/bench_C3.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_C3.json').read().strip().splitlines()[-1]); r=d['roofline']['ranked_us_per_step']; print('C3', d['value'], d['ms_per_step'], r)"
