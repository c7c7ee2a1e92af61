#!/bin/bash
# MHA probability-image swizzle: parity tests, isolated timing, LDS bank-conflict counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6mha
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py tests/test_attvis_gpu.py tests/test_greedy_gpu.py tests/test_beam_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 120 python tools/mha_bench.py 30 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
cat $O/bench.txt
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d $O/pmc -o run -- python tools/mha_bench.py 5 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r6mha/pmc/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    if "mha" in k:
        print(k, {c: int(x) for c, x in v.items()}, "conflict/inst %.3f" % (v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_INSTS_LDS"])))
PY
