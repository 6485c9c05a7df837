set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_tests.sh r03k "tests/test_gpu_kernels.py tests/test_gpu_models.py" "attention or multi_unit or persistent or latent" || exit 1
O=gpurun_out/r03k_lat_gemm.txt
GB_TAG=new timeout -k 10 120 python -u tools/gemm_latent_bench.py > $O 2>&1 || { tail -5 $O; exit 1; }
grep -v amdgpu.ids $O
timeout -k 10 300 python -u bench.py --config latent_vit --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r03k_lat.txt 2>&1 || { tail -5 gpurun_out/r03k_lat.txt; exit 1; }
tail -1 gpurun_out/r03k_lat.txt | cut -c1-250
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03k_latp -o run \
  -- python3 bench.py --config latent_vit --steps 20 --warmup 5 --probe-steps 0 --no-cpu-baseline > gpurun_out/r03k_latp.log 2>&1 || { tail -5 gpurun_out/r03k_latp.log; exit 1; }
python3 tools/prof_csv_summary.py gpurun_out/r03k_latp/run_kernel_stats.csv 28 40 > gpurun_out/r03k_lat_summary.txt; head -32 gpurun_out/r03k_lat_summary.txt
