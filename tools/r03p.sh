set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03p "tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_graph.py" "wgrad or latent or image_vit_48 or epoch or reference or graph" || exit 1
for cfg in latent_vit image_vit_48 hybrid_latent_vit expression_aware_vit; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03p_$cfg.txt 2>&1 || { tail -5 gpurun_out/r03p_$cfg.txt; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r03p_$cfg.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_mfma_frac"], d["final_loss"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03p_latp -o run \
  -- python3 bench.py --config latent_vit --steps 20 --warmup 5 --probe-steps 0 --no-cpu-baseline > gpurun_out/r03p_latp.log 2>&1 || { tail -5 gpurun_out/r03p_latp.log; exit 1; }
python3 tools/prof_csv_summary.py gpurun_out/r03p_latp/run_kernel_stats.csv 28 40 > gpurun_out/r03p_lat_summary.txt; head -25 gpurun_out/r03p_lat_summary.txt
