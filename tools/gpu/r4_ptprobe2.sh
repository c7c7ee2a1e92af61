#!/bin/bash
# Round 4: the persistent-tile loop skeleton (no MFMA, no DMA) with and without barrier / waits
set -o pipefail
O=gpurun_out/r4ptprobe; mkdir -p $O
: > $O/probe2.txt
for v in "neither:IMGCAP_PT_DBG=3" "nobar:IMGCAP_PT_DBG=7" "nowait:IMGCAP_PT_DBG=11" "none:IMGCAP_PT_DBG=15" "mfma_only_nobar:IMGCAP_PT_DBG=6"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 120 python -u tools/pt_probe.py $tag >> $O/probe2.txt 2>&1 || { cat $O/probe2.txt; exit 1; }
done
cat $O/probe2.txt
