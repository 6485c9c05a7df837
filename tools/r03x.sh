set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03x.txt; : > $O
export GB_ONLY=wgrad,wgrad_out,wgrad_qkv
GB_TAG=auto timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
for t in 64 128 512; do
FERVIT_GEMM_SPLIT_T256=$t GB_TAG=t256-$t timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
done
for c in 4 7 6; do
FERVIT_GEMM_CFG=$c GB_TAG=cfg$c timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
done
grep -v amdgpu.ids $O
