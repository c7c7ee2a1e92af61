#!/bin/bash
# Round 4: where the persistent-tile GEMM's time goes (MFMA-only / DMA-only / one block per tile)
set -o pipefail
O=gpurun_out/r4ptprobe; mkdir -p $O
: > $O/probe.txt
for v in "full:" "nomfma:IMGCAP_PT_DBG=1" "nodma:IMGCAP_PT_DBG=2" "neither:IMGCAP_PT_DBG=3" "grid:IMGCAP_PT_GRID=1" "grid_nodma:IMGCAP_PT_GRID=1 IMGCAP_PT_DBG=2"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 120 python -u tools/pt_probe.py $tag >> $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
done
cat $O/probe.txt
