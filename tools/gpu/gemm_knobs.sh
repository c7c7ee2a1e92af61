# GEMM census of a config under the LDS-DMA tile knobs (IMGCAP_GEMM_ORDER x IMGCAP_GLDS64_STAGES)
# usage: bash tools/gpu/gemm_knobs.sh CFG "ORDER:S64 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${1:-C2}; shift
for v in ${@:-0:2 1:2 0:3 1:3 0:4 1:4}; do
  o=${v%%:*}; s=${v#*:}
  IMGCAP_GEMM_ORDER=$o IMGCAP_GLDS64_STAGES=$s timeout -k 10 300 python tools/gemm_census.py $CFG > gpurun_out/knob_${CFG}_$o$s.txt 2>&1 || { tail -20 gpurun_out/knob_${CFG}_$o$s.txt; exit 1; }
  echo "order=$o s64=$s: $(sed -n 2p gpurun_out/knob_${CFG}_$o$s.txt)"
done
