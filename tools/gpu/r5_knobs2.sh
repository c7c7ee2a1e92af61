#!/bin/bash
# C2 / C5: switch alternates against the defaults, same box, two rounds
set -o pipefail
O=gpurun_out/r5knobs2; rm -rf $O; mkdir -p $O
for r in 1 2; do
for v in "NONE=1" "IMGCAP_LSTM_YS=2" "IMGCAP_LSTM_YS=4" "IMGCAP_LSTM_XS=3" "IMGCAP_MLP_RES=0" "IMGCAP_GEMM_PT=0"; do
  env $v timeout -k 10 300 python -u bench.py --config C2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "C2 $v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done
for v in "NONE=1" "IMGCAP_GEMM_PT=0" "IMGCAP_GEMM256=0" "IMGCAP_DW_CP_R=1" "IMGCAP_COLSUM=1"; do
  env $v timeout -k 10 300 python -u bench.py --config C5 --steps 40 --warmup 5 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "C5 $v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done; done
