set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 1 2 3; do
FERVIT_WG_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread -k wgrad_group > gpurun_out/r03o_t$v.txt 2>&1 || { tail -20 gpurun_out/r03o_t$v.txt; exit 1; }
tail -1 gpurun_out/r03o_t$v.txt
done
O=gpurun_out/r03o.txt; : > $O
export GB_ONLY=wgrad_group
for v in 0 1 2 3; do for sp in 1 2; do
FERVIT_WG_VARIANT=$v FERVIT_WG_SPLITS=$sp GB_TAG=v$v-sp$sp timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || { tail -5 $O; exit 1; }
done; done
grep -v amdgpu.ids $O | grep -v "layer sum"
