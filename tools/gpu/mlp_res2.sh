# resident-weight C=96 MLP variants (kernel bench): tm = 16-row slabs per unit, gelu 1 = sigmoid form
set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench
for v in "0 2 1" "0 1 1" "0 2 0"; do
set -- $v
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize -munsafe-fp-atomics -DMLP_RES_GRAB=$1 -DMLP_RES_TM=$2 -DMLP_RES_GELU=$3 -DMLP_TAG="\"grab$1_tm$2_gelu$3\"" mlp_bench.hip -o /tmp/mlp_v 2>/dev/null || exit 1
timeout -k 5 60 /tmp/mlp_v || exit 1
done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize -munsafe-fp-atomics -DMLP_RES_GRAB=0 -DMLP_STAMPS -DMLP_RES_STAMPS -DMLP_TAG="\"st\"" mlp_bench.hip -o /tmp/mlp_st || exit 1
timeout -k 5 60 /tmp/mlp_st || exit 1
