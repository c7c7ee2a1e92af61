#!/bin/bash
# MHA rewrite: decoder suites, C3 bench, kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5mha; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_transformer_gpu.py tests/test_attvis_gpu.py tests/test_beam_gpu.py tests/test_greedy_gpu.py tests/test_testpy_gpu.py tests/test_train_step_gpu.py tests/test_trainer_fullsize_gpu.py tests/test_headline_bf16_gpu.py tests/test_checkpoint_gpu.py > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -le 1 ] || exit $rc
for c in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b_$c.txt 2>$O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
  echo "$c $(python -c "import json; d=json.loads(open('$O/b_$c.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config C3 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r5mha/prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:24]:
    print(f'{r["Name"][:90]:90s} n={r["Calls"]:>6s} avg={float(r["AverageNs"])/1e3:7.2f}us min={float(r["MinNs"])/1e3:7.2f} share={float(r["Percentage"]):5.2f}')
PY
