set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03r.txt; : > $O
export GB_ONLY=fc2_fwd,fc1_dgrad,qkv_dgrad
for t in 256 304; do
FERVIT_GEMM_SPLIT_T128=$t GB_TAG=t$t-sep timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || exit 1
FERVIT_SPLITK_INLAUNCH=1 FERVIT_GEMM_SPLIT_T128=$t GB_TAG=t$t-inl timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || exit 1
FERVIT_GEMM_CFG=2 FERVIT_SPLITK_INLAUNCH=1 FERVIT_GEMM_SPLIT_T128=$t GB_TAG=cfg2-t$t-inl timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || exit 1
done
unset GB_ONLY
grep -v amdgpu.ids $O | grep -v "layer sum"
bash tools/attn_pmc.sh r03r > gpurun_out/r03r_pmc.log 2>&1 || { tail -5 gpurun_out/r03r_pmc.log; exit 1; }
cat gpurun_out/pmc_r03r_summary.txt
