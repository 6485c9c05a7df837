set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03q "tests/test_gpu_kernels.py tests/test_gpu_models.py" "gemm or linear or wgrad or many_tiles or every_tile or vit_base or latent" || exit 1
O=gpurun_out/r03q.txt; : > $O
GB_ONLY=wgrad GB_TAG=inlaunch timeout -k 10 100 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
FERVIT_SPLITK_SEPARATE=1 GB_ONLY=wgrad GB_TAG=separate timeout -k 10 100 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
export GB_ONLY=fc2_fwd,fc1_dgrad,qkv_dgrad,out_fwd,qkv_fwd
for t in 256 512; do
FERVIT_GEMM_SPLIT_T128=$t GB_TAG=lat-t$t timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || exit 1
FERVIT_SPLITK_SEPARATE=1 FERVIT_GEMM_SPLIT_T128=$t GB_TAG=lat-t$t-sep timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || exit 1
done
unset GB_ONLY
grep -v amdgpu.ids $O | grep -v "layer sum"
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r03q_bench.txt 2>&1 || { tail -5 gpurun_out/r03q_bench.txt; exit 1; }
tail -1 gpurun_out/r03q_bench.txt | cut -c1-200
FERVIT_SPLITK_SEPARATE=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r03q_bench_sep.txt 2>&1 || { tail -5 gpurun_out/r03q_bench_sep.txt; exit 1; }
tail -1 gpurun_out/r03q_bench_sep.txt | cut -c1-200
