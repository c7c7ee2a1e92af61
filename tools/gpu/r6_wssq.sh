#!/bin/bash
# SQ counters of the stage-3 GEMM (12544 x 1536 x 384 + GELU): the LDS-staged plan vs the ws kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6wssq; rm -rf $O; mkdir -p $O
S="${SHAPE:-12544 1536 384}"
for cfg in "0:" "1:" "1:IMGCAP_WS_STG=1" "1:IMGCAP_WS_PIPE=1"; do
  mode=${cfg%%:*}; envv=${cfg#*:}; tag=m${mode}$(echo "$envv" | tr -dc 'A-Z' | tail -c 5)
  i=0
  for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 60 env $envv rocprofv3 --pmc $set --output-format csv -d $O/${tag}p$i -o run -- python tools/ws_one.py $S $mode 5 gelu > $O/${tag}p$i.log 2>&1 || { tail -5 $O/${tag}p$i.log; exit 1; }
  done
  python tools/sq_summary.py $O/sq_$tag.json $O/${tag}p1 $O/${tag}p2 > /dev/null
  python - $O/sq_$tag.json $tag <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "gemm" not in k:
        continue
    w = v.get("SQ_WAVES", 1)
    keys = ["SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT"]
    print(f"{sys.argv[2]} {k[:50]}: waves {w} mfma_busy {v.get('mfma_busy')} " + " ".join(f"{c[3:]}={v.get(c, 0) / w:.0f}" for c in keys))
PY
done
