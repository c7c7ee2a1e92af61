# instruction-cache / wait counters of the persistent LSTM forward (microbench lstm)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lp_pmc
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/lp_pmc/a -o run -- python tools/microbench.py lstm > gpurun_out/lp_pmc/a.log 2>&1 || { tail -20 gpurun_out/lp_pmc/a.log; exit 1; }
f=$(find gpurun_out/lp_pmc/a -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:70]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "persist" in k or "attn_fwd" in k or "gate_cell" in k:
        print(k, {c: round(v / max(1, n[(k, c)])) for c, v in d.items()})
PY
