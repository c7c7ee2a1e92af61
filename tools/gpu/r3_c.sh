# round 3: C2 / C3 per-call kernel tables (roofline dump) and a C2 kernel-trace timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
IMGCAP_ROOFLINE_TABLE=$O/C2_table.json timeout -k 10 300 python -u bench.py --config C2 --steps 30 --no-cpu-baseline > $O/c2.log 2>&1 || { tail -30 $O/c2.log; exit 1; }
IMGCAP_ROOFLINE_TABLE=$O/C3_table.json timeout -k 10 300 python -u bench.py --config C3 --steps 30 --no-cpu-baseline > $O/c3.log 2>&1 || { tail -30 $O/c3.log; exit 1; }
IMGCAP_ROOFLINE_TABLE=$O/C4_table.json timeout -k 10 300 python -u bench.py --config C4 --steps 30 --no-cpu-baseline > $O/c4.log 2>&1 || { tail -30 $O/c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --config C2 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -30 $O/trace.log; exit 1; }
python tools/trace_path.py $(ls $O/trace/*kernel_trace.csv | head -1) --last 8000 > $O/trace_summary.txt 2>&1
head -60 $O/trace_summary.txt
