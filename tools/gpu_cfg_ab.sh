# Tile-config A/B on the ViT-B shapes, with and without the epilogue (FERVIT_GEMM_DBG=4 = main loop only).
# usage: bash tools/gpu_cfg_ab.sh <tag> "<cfgs>" [GB_ONLY filter]
set -o pipefail
TAG=${1:-ab}; CFGS=${2:-"8 11"}; export GB_ONLY=${3:-}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "tile_config" > gpurun_out/cfg_t_$TAG.txt 2>&1 || { tail -30 gpurun_out/cfg_t_$TAG.txt; exit 1; }
tail -1 gpurun_out/cfg_t_$TAG.txt
cd tools
for c in $CFGS; do FERVIT_GEMM_CFG=$c timeout -k 10 150 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee ../gpurun_out/cfg_$TAG.txt
for c in $CFGS; do FERVIT_GEMM_DBG=4 FERVIT_GEMM_CFG=$c timeout -k 10 150 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/[noepi] /" || exit 1; done | tee -a ../gpurun_out/cfg_$TAG.txt
