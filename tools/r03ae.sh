set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03ae "tests/test_gpu_models.py tests/test_gpu_hybrid.py tests/test_gpu_train.py tests/test_gpu_ddp.py tests/test_gpu_rccl.py tests/test_gpu_graph.py" || exit 1
for cfg in latent_vit image_vit_48 hybrid_latent_vit expression_aware_vit; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03ae_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03ae_$cfg.txt; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r03ae_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_mfma_frac"], d["final_loss"])')"
done
