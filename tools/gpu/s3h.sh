set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/blaslt -o run -- python tools/probe/blaslt_names.py > gpurun_out/blaslt.log 2>&1 || { tail -5 gpurun_out/blaslt.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/blaslt/**/*kernel_trace.csv", recursive=True)[0]
seen = []
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "Cijk" in n or "gemm" in n.lower():
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        seen.append((n[:150], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Workgroup_Size_X", ""), d))
for s in seen:
    print(f"{s[3]:7.1f} us grid {s[1]} wg {s[2]} {s[0]}")
PY
timeout -k 10 240 python -u tools/probe/capture_bisect.py C4 split full2 > gpurun_out/bisect.log 2>&1; rc=$?
grep -v "^frame" gpurun_out/bisect.log | grep -v Warn | grep -E "^ok|bisect|Error" | head -12
exit $rc
