# Direct (register) vs LDS-staged GEMM epilogue: parity tests, then gemm_bench with each.
# usage: bash tools/gpu_epi.sh <tag> [pytest -k]
set -o pipefail
TAG=${1:-e}; K=${2:-"gemm or linear"}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "$K" > gpurun_out/epi_t_$TAG.txt 2>&1 || { tail -30 gpurun_out/epi_t_$TAG.txt; exit 1; }
tail -1 gpurun_out/epi_t_$TAG.txt
cd tools
for d in 0 16; do
  echo "== FERVIT_GEMM_DBG=$d"
  FERVIT_GEMM_DBG=$d timeout -k 10 150 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done | tee ../gpurun_out/epi_$TAG.txt
