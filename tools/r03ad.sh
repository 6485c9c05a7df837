set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03ad "tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_graph.py" "attention or multi_unit or persistent or vit or latent or graph or head_dropout" || exit 1
O=gpurun_out/r03ad_attn.txt; : > $O
for v in "A=1" "FERVIT_ATTN_MASK_INLINE=1" "A=1" "FERVIT_ATTN_MASK_INLINE=1"; do
echo "[$v]" >> $O; env $v timeout -k 10 120 python -u tools/attn_bench.py >> $O 2>&1 || exit 1
done
grep -v amdgpu.ids $O
for v in "A=1" "FERVIT_ATTN_MASK_INLINE=1" "A=1" "FERVIT_ATTN_MASK_INLINE=1"; do
  env $v timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-traffic --probe-steps 1 > gpurun_out/r03ad.txt 2>&1 || { tail -5 gpurun_out/r03ad.txt; exit 1; }
  echo "[$v] $(tail -1 gpurun_out/r03ad.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms_median"], d["final_loss"])')"
done
