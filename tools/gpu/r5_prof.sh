#!/bin/bash
# kernel stats of the C3 step: pipelined (the bench) and unpipelined (no encoder beside the decoder)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5prof; rm -rf $O; mkdir -p $O
for v in pipe nopipe; do
  extra=""; [ $v = nopipe ] && extra="--no-pipeline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python bench.py --config ${CFG:-C3} --steps 30 --warmup 5 --no-cpu-baseline --no-roofline $extra > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  tail -1 $O/$v.log
done
python - <<'PY'
import csv, glob
for v in ("pipe", "nopipe"):
    f = glob.glob(f"gpurun_out/r5prof/{v}/**/run_kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"== {v}: total kernel ns {tot:.0f}")
    for r in rows[:28]:
        print(f'{r["Name"][:90]:90s} n={r["Calls"]:>6s} avg={float(r["AverageNs"])/1e3:7.2f}us min={float(r["MinNs"])/1e3:7.2f} share={float(r["Percentage"]):5.2f}')
PY
