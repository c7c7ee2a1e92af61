#!/bin/bash
# C3 schedule probes: pipelined graph with / without the runtime's graph packet capture, the
# sequential schedule, and the kernel-trace timeline without packet capture.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4sched; mkdir -p $O
B="python bench.py --config C3 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline"
timeout -k 10 200 $B > $O/default.log 2>&1 && tail -1 $O/default.log | cut -c1-140 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 $B > $O/nopacket.log 2>&1 && tail -1 $O/nopacket.log | cut -c1-140 &&
timeout -k 10 200 $B --no-pipeline > $O/seq.log 2>&1 && tail -1 $O/seq.log | cut -c1-140 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 bash tools/gpu/r4_trace.sh C3 > /dev/null && mv gpurun_out/trace_C3 $O/trace_nopacket &&
grep -A3 "=== step 13" $O/trace_nopacket/path.txt
