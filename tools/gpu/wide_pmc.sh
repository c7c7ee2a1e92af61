# round 3: wide MLP LDS counters (compute-only and full) at the C4 stage-3 shape
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wide
mkdir -p $O
for m in 2 0; do
  IMGCAP_WIDE_DBG=$m timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_INSTS_MFMA --output-format csv -d $O/pmc$m -o run -- python tools/mlp_wide_bench.py --only 2 --rounds 1 --reps 5 --fused-only > $O/pmc$m.log 2>&1 || { tail -5 $O/pmc$m.log; exit 1; }
  f=$(find $O/pmc$m -name "*counter_collection.csv" | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if "wide_kernel" not in r["Kernel_Name"]: continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(agg): print(f"  {k:34s} {agg[k] / max(1, n[k]):.4g} (avg over {n[k]} dispatch rows)")
PY
  rm -rf $O/pmc$m
done
