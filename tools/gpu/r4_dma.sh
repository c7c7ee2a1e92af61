#!/bin/bash
# Round 4: per-CU LDS-DMA / plain-load delivery rates (tools/kbench/dma_bench.hip)
set -o pipefail
O=gpurun_out/r4dma; mkdir -p $O
timeout -k 10 120 ./build/dma_bench > $O/dma.txt 2>&1; rc=$?; cat $O/dma.txt; exit $rc
