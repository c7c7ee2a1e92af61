#!/bin/bash
# SQ counters of one GEMM shape: the stream-tile kernel vs the LDS-staged plan
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5sq; rm -rf $O; mkdir -p $O
S="${SHAPE:-12544 384 1536}"
for mode in ${MODES:-0 4}; do
  i=0
  for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $O/m${mode}p$i -o run -- python tools/pt_one.py $S $mode 5 > $O/m${mode}p$i.log 2>&1 || { tail -5 $O/m${mode}p$i.log; exit 1; }
  done
  python tools/sq_summary.py $O/sq_m$mode.json $O/m${mode}p1 $O/m${mode}p2 > /dev/null
  python - $O/sq_m$mode.json $mode <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "gemm" not in k:
        continue
    w = v.get("SQ_WAVES", 1)
    keys = ["SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT"]
    print(f"mode {sys.argv[2]} {k[:60]}: waves {w} mfma_busy {v.get('mfma_busy')} " + " ".join(f"{c[3:]}={v.get(c, 0) / w:.0f}" for c in keys))
PY
done
