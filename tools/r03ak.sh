set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03ak "tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_hybrid.py tests/test_gpu_train.py" "wgrad or colsum or latent or image_vit_48 or hybrid or cfg4 or cfg5 or clip or epoch or linear or every_tile" || exit 1
O=gpurun_out/r03ak.txt; : > $O
GB_ONLY=wgrad_group GB_TAG=acquire-only timeout -k 10 120 python -u tools/gemm_latent_bench.py >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O | grep -v "layer sum"
for cfg in latent_vit image_vit_48 hybrid_latent_vit; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03ak_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03ak_$cfg.txt; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r03ak_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_mfma_frac"], d["final_loss"])')"
done
