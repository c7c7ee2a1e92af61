#!/bin/bash
# encoder-branch capture order of the pipelined step: start / interleave (C3 trace + bench)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5fork; rm -rf $O; mkdir -p $O
for f in ${FORKS:-swap start}; do
  IMGCAP_PIPE_FORK=$f bash tools/gpu/r4_trace.sh C3 > $O/trace_$f.txt 2>&1 || { tail -20 $O/trace_$f.txt; exit 1; }
  grep -E "wall|queue [0-9]|idle" $O/trace_$f.txt | head -6
  cp gpurun_out/trace_C3/path.txt $O/path_$f.txt
done
for c in C3 C4; do
  for f in ${FORKS:-swap start}; do
    IMGCAP_PIPE_FORK=$f timeout -k 10 300 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b_${c}_$f.txt 2>$O/b_${c}_$f.err || { tail -20 $O/b_${c}_$f.err; exit 1; }
    echo "$c $f $(python -c "import json; d=json.loads(open('$O/b_${c}_$f.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
  done
done
