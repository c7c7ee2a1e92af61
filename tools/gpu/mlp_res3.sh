set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -munsafe-fp-atomics -DMLP_RES_GRAB=0 -DMLP_STAMPS -DMLP_RES_STAMPS -DMLP_TAG="\"st\"" mlp_bench.hip -o /tmp/mlp_st || exit 1
timeout -k 5 60 /tmp/mlp_st || exit 1
