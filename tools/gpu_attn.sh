# Attention parity tests + microbenchmark (ViT-B/16 bs=256 shape). usage: bash tools/gpu_attn.sh <tag>
set -o pipefail
TAG=${1:-a}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "attention or model_matches" > gpurun_out/attn_t_$TAG.txt 2>&1 || { tail -40 gpurun_out/attn_t_$TAG.txt; exit 1; }
tail -2 gpurun_out/attn_t_$TAG.txt
cd tools && timeout -k 10 120 python -u attn_bench.py 2>&1 | grep -v amdgpu.ids | tee ../gpurun_out/attn_b_$TAG.txt
