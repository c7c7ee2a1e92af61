#!/bin/bash
# eager pipelined C3 (--no-graph): the encoder stream CU-masked or not -- trace start of the decoder
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5cumask; rm -rf $O; mkdir -p $O
for m in 0 192; do
  IMGCAP_ENC_CUMASK=$m bash tools/gpu/r4_trace.sh C3 --no-graph > $O/trace_$m.txt 2>&1 || { tail -20 $O/trace_$m.txt; exit 1; }
  echo "mask $m"; grep -E "wall|queue [0-9]|idle" $O/trace_$m.txt | head -5
  cp gpurun_out/trace_C3/path.txt $O/path_$m.txt
  IMGCAP_ENC_CUMASK=$m timeout -k 10 300 python -u bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline --no-roofline --no-graph > $O/b_$m.txt 2>$O/b_$m.err || { tail -20 $O/b_$m.err; exit 1; }
  echo "C3 eager mask $m $(python -c "import json; d=json.loads(open('$O/b_$m.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
