# round 3: the bench with the per-call roofline (C2, C3), then the C5 artifact sequence that hung
# in round 2 (a FETCH_SIZE pass, then the 200-step bench with progress marks)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u bench.py --config C2 --steps 60 --cpu-seconds 5 > $O/c2.log 2>&1 || { tail -30 $O/c2.log; exit 1; }
tail -1 $O/c2.log | cut -c1-3000
timeout -k 10 300 python -u bench.py --config C3 --steps 60 --no-cpu-baseline > $O/c3.log 2>&1 || { tail -30 $O/c3.log; exit 1; }
tail -1 $O/c3.log | cut -c1-3000
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py --config C5 --steps 3 --warmup 2 --no-cpu-baseline > $O/fetch5.log 2>&1 || { tail -30 $O/fetch5.log; exit 1; }
IMGCAP_BENCH_PROGRESS=1 timeout -k 10 400 python -u bench.py --config C5 --no-cpu-baseline > $O/c5.log 2>&1 || { echo "c5 rc=$?"; tail -30 $O/c5.log; exit 1; }
tail -1 $O/c5.log | cut -c1-3000
