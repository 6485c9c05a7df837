set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03s "tests/test_gpu_kernels.py tests/test_gpu_models.py" "every_tile or epilogue_kinds or linear or latent or image_vit_48" || exit 1
O=gpurun_out/r03s.txt; : > $O
GB_TAG=auto timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || exit 1
FERVIT_GEMM_CFG=11 GB_TAG=cfg11 timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
for cfg in latent_vit image_vit_48 hybrid_latent_vit; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03s_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03s_$cfg.txt; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r03s_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_mfma_frac"], d["final_loss"])')"
done
O=gpurun_out/r03s_prio.txt; : > $O
export FERVIT_LIB=$PWD/fer-vit_amd/fervit/libfervit_exp.so GB_ONLY=gate,res_fc2,mul,store_qkv,plain_fc1,res_out
for rep in 1 2; do
GB_TAG=base$rep timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
FERVIT_GEMM_DBG=$((1 << 20)) GB_TAG=prio-hi$rep timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
FERVIT_GEMM_DBG=$((1 << 21)) GB_TAG=prio-lo$rep timeout -k 10 200 python -u tools/gemm_cases_bench.py >> $O 2>&1 || exit 1
done
grep -v amdgpu.ids $O
