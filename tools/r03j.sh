set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03j_lat_split.txt; : > $O
export GB_ONLY=fc2_fwd,fc1_dgrad,qkv_dgrad,qkv_wgrad,out_wgrad,fc1_wgrad,fc2_wgrad
for c in 2 3 6 7; do for t in 128 256 512 1024; do
  FERVIT_GEMM_CFG=$c FERVIT_GEMM_SPLIT_T128=$t GB_TAG=cfg$c-t$t timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || { tail -5 $O; exit 1; }
done; done
grep -v amdgpu.ids $O
