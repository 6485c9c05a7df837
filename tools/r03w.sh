set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03w.txt; : > $O
export FERVIT_LIB=$PWD/fer-vit_amd/fervit/libfervit_exp.so GB_ONLY=gate,res_fc2,mul,store_qkv,plain_fc1,res_out,res_qkvd
for rep in 1 2; do for gs in 0 1 2 3; do
FERVIT_GEMM_DBG=$((gs << 22)) GB_TAG=grp$gs-$rep timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O
