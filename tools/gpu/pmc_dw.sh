set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-include-regex "dwconv7_kernel|cnblock_mlp" --output-format csv -d gpurun_out/pmc_dw -o run -- python tools/microbench.py mlpdw > gpurun_out/pmc_dw.log 2>&1 || { tail -20 gpurun_out/pmc_dw.log; exit 1; }
find gpurun_out/pmc_dw -name "*.csv" | head
