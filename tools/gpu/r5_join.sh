#!/bin/bash
# interleaved encoder capture with join edges (graph submission order): trace + C3 bench
# (the interleaved capture with IMGCAP_PIPE_FORK=interleave / IMGCAP_PIPE_JOIN / IMGCAP_PIPE_TICK was measured
# slower and removed -- DESIGN 2b; the script is kept as the record of the run)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5join; rm -rf $O; mkdir -p $O
for v in "start 0 3" "interleave 1 3" "interleave 1 5" "interleave 2 3" "interleave 0 3"; do
  set -- $v
  export IMGCAP_PIPE_FORK=$1 IMGCAP_PIPE_JOIN=$2 IMGCAP_PIPE_TICK=$3
  bash tools/gpu/r4_trace.sh C3 > $O/trace_$1_$2_$3.txt 2>&1 || { tail -20 $O/trace_$1_$2_$3.txt; exit 1; }
  echo "== $v"; grep -E "wall|queue [0-9]" $O/trace_$1_$2_$3.txt | head -5
  timeout -k 10 300 python -u bench.py --config C3 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "C3 $v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
