set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03l.txt; : > $O
export GB_ONLY=fc1_wgrad,fc1_wgrad_kk,out_wgrad,qkv_wgrad
for c in 3 2; do for t in 128 256 512; do
  FERVIT_GEMM_CFG=$c FERVIT_GEMM_SPLIT_T128=$t GB_TAG=cfg$c-t$t timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || { tail -5 $O; exit 1; }
done; done
grep -v amdgpu.ids $O | grep -v "layer sum"
