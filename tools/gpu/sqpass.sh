# SQ counter passes of a bench config -> profiles/<ROUND>_<CFG>_sq.json (tools/sq_summary.py)
# usage: bash tools/gpu/sqpass.sh CFG ROUND
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=$1; ROUND=${2:-r02}
O=gpurun_out/sq_$CFG
mkdir -p $O
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python bench.py --config $CFG --steps 3 --warmup 2 --no-cpu-baseline --no-graph > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python tools/sq_summary.py profiles/${ROUND}_${CFG}_sq.json $O/p1 $O/p2 $O/p3
