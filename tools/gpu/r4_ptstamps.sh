#!/bin/bash
# Round 4: depthwise / MX / PT tests after the variant pruning and the MX depthwise epilogue, then
# the persistent-tile GEMM skeleton probe + in-kernel stamps (diagnostic build)
set -o pipefail
O=gpurun_out/r4ptprobe; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dwconv_cp_gpu.py tests/test_mx_gpu.py tests/test_gemm_pt_gpu.py tests/test_kernels_gpu.py -k "dwconv or mx or pt" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/probe2.txt
for v in "neither:IMGCAP_PT_DBG=3" "nobar:IMGCAP_PT_DBG=7" "nowait:IMGCAP_PT_DBG=11" "none:IMGCAP_PT_DBG=15"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 120 python -u tools/pt_probe.py $tag >> $O/probe2.txt 2>&1 || { cat $O/probe2.txt; exit 1; }
done
grep -v amdgpu.ids $O/probe2.txt
: > $O/stamps.txt
for c in 2 4; do
  timeout -k 10 120 python -u tools/pt_stamps.py $c >> $O/stamps.txt 2>&1 || { cat $O/stamps.txt; exit 1; }
done
grep -v amdgpu.ids $O/stamps.txt
