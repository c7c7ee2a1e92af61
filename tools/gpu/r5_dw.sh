#!/bin/bash
# XCD-contiguous depthwise slots: parity, microbench, FETCH_SIZE, C3 / C4 bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5dw; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_encoder_gpu.py tests/test_dwconv_cp_gpu.py tests/test_encoder_train_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" $O/tests.log | head; exit 1; }
timeout -k 10 200 python -u tools/microbench.py dw > $O/dw.txt 2>&1 && grep -v amdgpu.ids $O/dw.txt || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python tools/microbench.py dw > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r5dw/fetch/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "dwconv7" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
        acc[(r["Kernel_Name"][:60], r.get("Grid_Size", ""))].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, f"FETCH {sum(v) / len(v) / 1024:.1f} MB/launch (KB units) x{len(v)}")
PY
for c in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "$c $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
