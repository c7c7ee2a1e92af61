set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/embp -o run -- python tools/probe/emb_time.py > gpurun_out/embp.log 2>&1 || { tail -20 gpurun_out/embp.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/embp/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "emb" in r["Name"]:
        print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
