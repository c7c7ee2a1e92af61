#!/bin/bash
# Round-4 baseline: per-GEMM census (ours vs hipBLASLt) at C3 / C4 and a short C3 bench.
set -o pipefail
mkdir -p gpurun_out/r4census
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_census.py C3 > gpurun_out/r4census/C3.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_census.py C4 > gpurun_out/r4census/C4.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config C3 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r4census/bench_C3.json 2> gpurun_out/r4census/bench_C3.err
